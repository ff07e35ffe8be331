"""LLMEngine: scheduler + native block manager + model runner + outputs.

``step()`` = schedule -> execute (one forward over decodes + prefill chunks)
-> sample -> update request state -> emit outputs, KV events and metrics.
The HTTP layer (``llmd_amd.serving``) drives ``step()`` from a dedicated
thread through ``AsyncEngine``.
"""
from __future__ import annotations

import logging
import time
from typing import Iterable, Optional

import torch

from llmd_amd import _rt_loader
from llmd_amd.parallel import symm as _symm
from llmd_amd.utils import markers

from .config import EngineConfig
from .metrics import EngineMetrics
from .model_runner import ModelRunner
from .request import Request, RequestOutput, SamplingParams, Status
from .scheduler import Scheduler, SchedulerOutput

log = logging.getLogger("llmd.engine")


def make_lora_manager(cfg: EngineConfig, runner: ModelRunner, driver: bool):
    from llmd_amd.parallel.comm import tp_broadcast_plan

    from .lora import LoRAManager

    n = max(cfg.sched.max_num_batched_tokens, cfg.cuda_graph_max_bs) + 64
    bc = tp_broadcast_plan if (driver and runner.tp_size > 1) else None
    mgr = LoRAManager(runner.model, max(1, cfg.max_loras), cfg.max_lora_rank, n, runner.device, broadcast=bc)
    runner.lora = mgr
    return mgr


class LLMEngine:
    def __init__(self, cfg: EngineConfig, metrics: Optional[EngineMetrics] = None,
                 runner: Optional[ModelRunner] = None, capture_graphs: bool = True):
        self.cfg = cfg
        self.runner = runner or ModelRunner(cfg)
        nb = self.runner.profile_and_allocate() if self.runner.kv is None else self.runner.num_blocks
        rt = _rt_loader.rt()
        ev_on = bool(cfg.kv_events_config and cfg.kv_events_config.get("enable_kv_cache_events"))
        if self.runner.hybrid:
            from .hybrid_kv import HybridBlockManager

            self.bm = HybridBlockManager(rt, nb, self.runner.num_swa_blocks, cfg.cache.block_size,
                                         self.runner.max_window, cfg.cache.enable_prefix_caching,
                                         ev_on or bool(cfg.kv_offload_config), swa_events=bool(cfg.kv_offload_config))
        else:
            self.bm = rt.BlockManager(nb, cfg.cache.block_size, cfg.cache.enable_prefix_caching,
                                      ev_on or bool(cfg.kv_offload_config))
        self.connector = None
        if cfg.kv_transfer_config:
            from llmd_amd.kvx.connector import make_connector

            self.connector = make_connector(cfg, self)
        self.sched = Scheduler(cfg, self.bm, self.connector)
        self.metrics = metrics or EngineMetrics(cfg.served_name, cfg.cache.block_size, nb,
                                                max_lora=cfg.max_loras if cfg.enable_lora else 0)
        self.event_sink = None  # set by serving.kv_events.KVEventPublisher
        self.offload = None
        if cfg.kv_offload_config:
            from llmd_amd.kvcache.offload import HybridOffload, OffloadManager

            self.offload = HybridOffload(cfg, self) if self.runner.hybrid else OffloadManager(cfg, self)
            self.sched.offload = self.offload
        from llmd_amd.parallel import ep

        ep.set_backend(cfg.parallel.all2all_backend)
        self.dp_lockstep = ep.ep_active() and self.runner.mc.is_moe
        if self.dp_lockstep:
            from llmd_amd.parallel.state import get_state

            st = get_state()
            log.info("wide-EP: DP rank %d/%d, experts sharded over %d EP ranks (%s), lockstep steps",
                     st.dp_rank, st.dp_size, st.ep_size, ep.backend())
        self.last_global_idle = False
        self.lora = None
        if cfg.enable_lora:
            self.lora = make_lora_manager(cfg, self.runner, driver=True)
            for name, path in (cfg.lora_modules or {}).items():
                self.lora.load(name, path)
        if capture_graphs:
            self.runner.capture_graphs()
        self.paused = False
        self.step_count = 0
        self.last_step_empty = False
        self.last_num_tokens = 0
        # async scheduling: the launched step whose tokens are still on the device
        self._pending = None  # (SchedulerOutput, DeferredSample, t0)
        self.async_sched = bool(cfg.sched.async_scheduling and not self.dp_lockstep and self.runner.tp_size == 1
                                and self.connector is None)

    # ------------------------------------------------------------ API
    def add_request(self, request_id: str, prompt_token_ids: list[int],
                    params: Optional[SamplingParams] = None, priority: int = 0,
                    kv_transfer_params: Optional[dict] = None, lora_id: int = 0,
                    arrival_time: Optional[float] = None, mm_inputs: Optional[list] = None) -> Request:
        if params is not None and params.logit_bias:
            params.check_vocab(self.cfg.model_config.vocab_size)
        r = Request(request_id, list(prompt_token_ids), params or SamplingParams(), priority=priority,
                    kv_transfer_params=kv_transfer_params, lora_id=lora_id, mm_inputs=mm_inputs or None)
        if arrival_time is not None:
            r.arrival_time = arrival_time
        self.sched.add_request(r)
        self.metrics.on_arrival(r)
        return r

    def abort(self, request_id: str):
        r = self.sched.abort(request_id)
        if r is not None:
            self.metrics.on_finish(r)

    def has_unfinished(self) -> bool:
        return self.sched.has_work() or self._pending is not None

    def block_tables(self, so: SchedulerOutput) -> dict[int, list[int]]:
        full = {sr.req.seq_id: self.bm.block_table(sr.req.seq_id) for sr in so.all()}
        if self.runner.hybrid:
            from .hybrid_kv import HybridTables

            return HybridTables(full, {sr.req.seq_id: self.bm.block_table_swa(sr.req.seq_id) for sr in so.all()})
        return full

    def step(self) -> list[RequestOutput]:
        # asleep, or woken from level 2 with the trainer's weights not yet sent:
        # new requests queue until the weights are real again
        if self.paused or self.sleeping or self.weights_pending:
            return self.drain()
        if self.async_sched:
            return self._step_async()
        if self.connector is not None:
            self.connector.tick()
        t0 = time.monotonic()
        with markers.range("llmd.schedule"):
            so = self.sched.schedule()
        if self.connector is not None and self.runner.tp_size > 1:
            self.connector.flush_tp()
        if self.lora is not None:
            nm = self.lora.name_of
            self.metrics.set_lora(sorted({nm(r.lora_id) for r in self.sched.running if r.lora_id} - {None}),
                                  sorted({nm(r.lora_id) for r in self.sched.waiting if r.lora_id} - {None}))
        err_outs = self._error_outputs()
        self.last_step_empty = so.empty
        self.last_num_tokens = so.num_tokens
        if self.dp_lockstep:
            return self._lockstep_step(so, err_outs, t0)
        if so.empty:
            self._flush_events()
            return err_outs
        if self.offload is not None:
            self.offload.before_step(so)
        sampled = self.runner.execute(so, self.block_tables(so))
        with markers.range("llmd.update"):
            return self._finish_step(so, sampled, err_outs, t0)

    # ------------------------------------------------------------ async scheduling
    def drain(self) -> list[RequestOutput]:
        """Outputs of the step still in flight (async scheduling), or []: called before
        anything that must see settled request state (pause, sleep, weight updates)."""
        pend, self._pending = self._pending, None
        return self._resolve(*pend) if pend is not None else []

    def _needs_settled(self, so) -> bool:
        """Steps whose planning reads output-token VALUES must wait for the step in flight:
        penalties / logit bias / min-p, embeddings, and a recompute chunk that re-reads a
        placeholder (a request preempted while its last token was in flight)."""
        for sr in so.decodes:
            sp = sr.req.params
            if sp.penalized or sp.embed:
                return True
        for sr in so.prefills:
            r = sr.req
            if r.params.penalized or r.params.embed or (r.async_pending and sr.start + sr.num_new_tokens >= r.num_tokens):
                return True
        return False

    def _step_async(self) -> list[RequestOutput]:
        """schedule N+1 (state advanced over step N's placeholders) -> launch N+1 (its decode
        inputs gathered on the device from N's samples) -> wait for N's tokens (N+1 is queued
        behind N, so the GPU never idles on the host) -> emit N's outputs. A request whose
        last token is in flight is not scheduled again; one stopped by EOS / a stop token
        costs one discarded row in the step launched before its token was seen."""
        t0 = time.monotonic()
        with markers.range("llmd.schedule"):
            so = self.sched.schedule()
        if self.lora is not None:
            nm = self.lora.name_of
            self.metrics.set_lora(sorted({nm(r.lora_id) for r in self.sched.running if r.lora_id} - {None}),
                                  sorted({nm(r.lora_id) for r in self.sched.waiting if r.lora_id} - {None}))
        outs = self._error_outputs()
        self.last_step_empty = so.empty
        self.last_num_tokens = so.num_tokens
        if so.empty:
            outs += self.drain()
            if self._pending is None and not outs:
                self._flush_events()
            return outs
        if self._pending is not None and self._needs_settled(so):
            outs += self.drain()
        if self.offload is not None:
            self.offload.before_step(so)
        prev = self._pending[1] if self._pending is not None else None
        handle = self.runner.execute(so, self.block_tables(so), prev=prev, defer=True)
        if self._pending is not None:
            with markers.range("llmd.update"):
                outs += self.drain()
        self.sched.advance(so, set(handle.seq_ids))
        self._pending = (so, handle, t0)
        return outs

    def _resolve(self, so, handle, t0) -> list[RequestOutput]:
        sampled = handle.host()
        _symm.check_health("emitting step %d" % self.step_count)
        touched = self.sched.resolve(so, sampled)
        return self._outputs(so, touched, [], t0)

    # ------------------------------------------------------------ DP lockstep
    def _lockstep_step(self, so, err_outs, t0) -> list[RequestOutput]:
        """Wide-EP (DP attention + EP MoE): every rank runs a forward
        whenever ANY rank has work - idle ranks a dummy one - with agreed shapes:
        all-decode steps replay the bucket of the largest decode batch, steps with
        a prefill anywhere run eager with MoE rows padded to the largest step."""
        import torch.distributed as dist

        from llmd_amd.parallel import ep
        from llmd_amd.parallel.state import get_state

        v = torch.tensor([so.num_tokens, int(bool(so.prefills)), len(so.decodes)], dtype=torch.int64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=get_state().cpu_group)
        t_max, any_prefill, nd_max = v.tolist()
        self.last_global_idle = t_max == 0
        if t_max == 0:
            self._flush_events()
            return err_outs
        pc = self.cfg.parallel
        if self._use_dbo(t_max, bool(any_prefill)):
            # dual-batch overlap. Decode-only: two micro-batches of ceil(t_max/2) MoE
            # rows on every rank, or bucket/2 rows when the step replays a captured
            # dual-batch graph. With prefills the chunks are not split, so a half
            # may hold up to t_max rows.
            dbo_b = None if any_prefill else self.runner.dbo_bucket(t_max)
            ep.set_step_rows(dbo_b // 2 if dbo_b else (t_max if any_prefill else (t_max + 1) // 2))
            if so.empty:
                self.runner.execute_dbo(None, {}, bucket=dbo_b)
                self.runner.eplb_tick()
                self._flush_events()
                return err_outs
            if self.offload is not None:
                self.offload.before_step(so)
            sampled = self.runner.execute_dbo(so, self.block_tables(so), bucket=dbo_b)
            self.runner.eplb_tick()
            return self._finish_step(so, sampled, err_outs, t0)
        bucket = None
        if not any_prefill and self.runner.graphs:
            b = self.runner._bucket(max(nd_max, 1))
            bucket = b if b in self.runner.graphs else None
        ep.set_step_rows(0 if bucket is not None else t_max)
        if so.empty:
            self.runner.execute_dummy(bucket)
            self.runner.eplb_tick()
            self._flush_events()
            return err_outs
        if self.offload is not None:
            self.offload.before_step(so)
        sampled = self.runner.execute(so, self.block_tables(so), force_eager=bucket is None, bucket=bucket)
        self.runner.eplb_tick()
        return self._finish_step(so, sampled, err_outs, t0)

    def _use_dbo(self, t_max: int, any_prefill: bool) -> bool:
        """Same decision on every EP rank (inputs are group-wide maxima). On the
        GPU the micro-batches run on two streams, which needs the per-micro-batch
        symm EP channels (RCCL calls of one communicator are not interleaved
        across streams) and rows within the symm receive buffers."""
        pc = self.cfg.parallel
        if not pc.enable_dbo:
            return False
        thr = pc.dbo_prefill_token_threshold if any_prefill else pc.dbo_decode_token_threshold
        if t_max < thr:
            return False
        if not self.runner.is_gpu:
            return True
        from llmd_amd.parallel import symm

        sep = symm.ep()
        return symm.micro_batches() >= 2 and sep is not None and t_max <= sep.R_max

    def dp_has_unfinished(self) -> bool:
        """True while any DP rank of the EP group still has requests."""
        if not self.dp_lockstep:
            return self.has_unfinished()
        import torch.distributed as dist

        from llmd_amd.parallel.state import get_state

        v = torch.tensor([int(self.has_unfinished())], dtype=torch.int64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=get_state().cpu_group)
        return bool(v.item())

    def _finish_step(self, so, sampled, err_outs, t0) -> list[RequestOutput]:
        # a timed-out symm collective (stalled peer) makes this step's tokens garbage:
        # fail loudly before any of them reaches a client (one host load, no sync)
        _symm.check_health("emitting step %d" % self.step_count)
        touched = self.sched.update(so, sampled)
        return self._outputs(so, touched, err_outs, t0)

    def _outputs(self, so, touched, err_outs, t0) -> list[RequestOutput]:
        dt = time.monotonic() - t0
        self.step_count += 1
        outs = err_outs
        for r in touched:
            o = RequestOutput(r.request_id, [r.output_token_ids[-1]], [r.output_logprobs[-1]],
                              r.status.finished, r.finish_reason, r.num_prompt_tokens,
                              len(r.output_token_ids), r.num_cached_tokens)
            if r.status.finished:
                o.kv_transfer_params = r.extra.get("kv_transfer_params_out")
                o.embedding = r.extra.get("embedding")
                self.metrics.on_finish(r)
            outs.append(o)
        self.metrics.on_step(so, touched, dt, self.sched.num_running, self.sched.num_waiting,
                             self.bm.usage(), self.bm.prefix_stats())
        self._flush_events()
        return outs

    def _error_outputs(self) -> list[RequestOutput]:
        outs = []
        for r in self.sched.errored:
            outs.append(RequestOutput(r.request_id, [], [], True, r.finish_reason, r.num_prompt_tokens,
                                      len(r.output_token_ids), r.num_cached_tokens))
            self.metrics.on_finish(r)
        self.sched.errored.clear()
        return outs

    def _flush_events(self):
        evs = self.bm.take_events() if (self.offload is not None or self.event_sink is not None) else []
        if self.offload is not None:
            self.offload.on_block_events(evs)
            if hasattr(self.offload, "on_swa_events"):
                self.offload.on_swa_events(self.bm.take_swa_events())
            self.offload.after_step()
            evs = list(evs) + self.offload.take_events()
        if self.event_sink is not None and evs:
            self.event_sink(evs)

    # ------------------------------------------------------------ offline helpers
    def generate(self, prompts: Iterable[list[int]], params: SamplingParams,
                 lora_ids: Optional[list[int]] = None) -> list[Request]:
        reqs = []
        for i, p in enumerate(prompts):
            reqs.append(self.add_request(f"gen-{self.step_count}-{i}-{time.monotonic_ns()}", p, params,
                                         lora_id=lora_ids[i] if lora_ids else 0))
        while self.has_unfinished():
            self.step()
        return reqs

    def shutdown(self):
        """Release TP followers (their loop exits) and the KV transfer agent."""
        if getattr(self, "_shut", False):
            return
        self._shut = True
        if self.runner.tp_size > 1:
            from .tp_worker import stop_followers

            stop_followers()
        if self.connector is not None and hasattr(self.connector, "close"):
            self.connector.close()

    def reset_prefix_cache(self):
        self.bm.reset_prefix_cache()
        self._flush_events()

    # ------------------------------------------------------------ RL weight sync / sleep (M17)
    @property
    def weight_sync(self):
        ws = getattr(self.runner, "weight_sync", None)
        if ws is None:
            from llmd_amd.parallel.comm import tp_broadcast_plan

            from .weight_sync import WeightSync

            ws = WeightSync(self.runner, tp_broadcast_plan if self.runner.tp_size > 1 else None)
            self.runner.weight_sync = ws
        return ws

    def weight_sync_cmd(self, cmd: dict) -> dict:
        """init_group / update_from_group / update_from_disk / destroy_group /
        sleep / wake_up on every TP rank of this replica (engine/weight_sync.py).
        Cached prefixes were computed with the old weights (or lost in sleep):
        the prefix cache is reset after every weight change."""
        op = cmd["op"]
        if op == "sleep" and self.has_unfinished():
            raise RuntimeError("cannot sleep with requests in flight (pause and drain first)")
        if op == "sleep" and self.connector is not None:
            raise RuntimeError("P/D engines cannot sleep: peers hold mappings of the KV pool")
        if self.weight_sync.sleeping and op not in ("wake_up", "sleep", "init_group", "destroy_group"):
            # level 2 woke up with uninitialised weights: the trainer sends them after wake_up
            raise RuntimeError("engine is asleep: wake_up first")
        if op == "sleep" and self.offload is not None and not self.weight_sync.sleeping:
            # the offloader holds the pool (and staging copies of it): let go first,
            # or the pool stays allocated while sleep reports it freed
            self.offload.rebind(None)
        try:
            res = self.weight_sync.apply(cmd)
        except BaseException:
            if op == "sleep" and self.offload is not None and not self.weight_sync.sleeping:
                self.offload.rebind(self.runner.kv)
            raise
        if op in ("update_from_group", "update_from_disk", "sleep", "wake_up"):
            self.reset_prefix_cache()
        if self.offload is not None:
            if op in ("update_from_group", "update_from_disk"):
                self.offload.invalidate(self.weight_sync.weights_id)  # offloaded KV is of the old weights
            elif op == "wake_up":
                self.offload.rebind(self.runner.kv)
        return res

    @property
    def sleeping(self) -> int:
        ws = getattr(self.runner, "weight_sync", None)
        return ws.sleeping if ws is not None else 0

    @property
    def weights_pending(self) -> bool:
        ws = getattr(self.runner, "weight_sync", None)
        return ws.weights_pending if ws is not None else False
