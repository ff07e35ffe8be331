"""Model runner: owns the model, the paged KV cache and the per-step execution.

KV cache: one tensor ``[L, num_blocks, 2, Hkv, block_size, D]`` (layer-major):
per-layer views ``kv[l, :, 0]`` / ``kv[l, :, 1]`` are contiguous pools, which
is what the attention kernels stream. A block-major layout (one block of
every layer contiguous, a single DMA per block for P/D and offload) cost the
decode kernel 5-11 % (203-208 vs 219-227 us per 70B layer at batch 64 ctx
5000, profiles/attn_decode_layout.txt): a sequence's blocks of one layer then
sit 20 MB apart across a 100+ GB range. Transfers instead move a block as 2 L
per-layer segments (kvx copy kernel segment lists, offload gathers).

Hybrid KV cache (engine/hybrid_kv.py; models with sliding-window layers):
the full-attention layers keep ``kv`` ([L_full, num_blocks, ...]) and the
windowed layers get their own small pool ``kv_swa`` ([L_swa, num_swa_blocks,
...]) with separate block tables and slot mappings (``AttnMeta.swa``).

Decode-only steps replay a captured hipGraph per batch bucket:
all inputs live in static device buffers, padded rows have ``slot = -1`` and
``seq_len = 1`` so they neither write the cache nor read past it. Mixed
steps (chunked prefill + decodes) run eagerly.
"""
from __future__ import annotations

import dataclasses
import logging
import math
import os
import time
from typing import Optional

import numpy as np
import torch

from llmd_amd.kvx.agent import p2p_step_guard
from llmd_amd import ops
from llmd_amd.models import build_model
from llmd_amd.parallel.comm import tp_broadcast_plan, tp_min_int
from llmd_amd.parallel.state import get_state
from llmd_amd.utils import markers

from .attn_meta import AttnMeta
from .config import EngineConfig
from .scheduler import ScheduledReq, SchedulerOutput

log = logging.getLogger("llmd.runner")


class DeferredSample:
    """A step's sampled tokens still on the device (async scheduling): the ids stay there
    for the next step's decode inputs; a non-blocking copy to pinned host memory plus an
    event let ``host()`` wait for exactly this step, not for the step launched after it."""

    __slots__ = ("ids", "lp", "seq_ids", "row_of", "_h_ids", "_h_lp", "_ev")

    def __init__(self, ids, lp, seq_ids, gpu: bool):
        self.ids, self.lp, self.seq_ids = ids, lp, seq_ids
        self.row_of = {s: i for i, s in enumerate(seq_ids)}
        self._ev = None
        if gpu and ids is not None:
            self._h_ids = torch.empty(ids.shape, dtype=ids.dtype, pin_memory=True)
            self._h_ids.copy_(ids, non_blocking=True)
            self._h_lp = None
            if lp is not None:
                self._h_lp = torch.empty(lp.shape, dtype=lp.dtype, pin_memory=True)
                self._h_lp.copy_(lp, non_blocking=True)
            self._ev = torch.cuda.Event()
            self._ev.record()
        else:
            self._h_ids, self._h_lp = ids, lp

    @classmethod
    def empty(cls) -> "DeferredSample":
        return cls(None, None, [], False)

    def host(self) -> dict[int, tuple[int, float]]:
        if not self.seq_ids:
            return {}
        if self._ev is not None:
            self._ev.synchronize()
        ids = self._h_ids.tolist()
        lp = self._h_lp.tolist() if self._h_lp is not None else [0.0] * len(ids)
        return {s: (int(ids[i]), float(lp[i])) for i, s in enumerate(self.seq_ids)}


def _mix64(z: int) -> int:
    z &= (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return (z ^ (z >> 31)) & ((1 << 63) - 1)


VMM_CHUNK = 2 << 30  # bytes per exportable KV-pool chunk


class ModelRunner:
    def __init__(self, cfg: EngineConfig, device: Optional[str] = None):
        self.cfg = cfg
        self.mc = cfg.model_config
        self.device = torch.device(device or cfg.device)
        if self.device.type == "cuda" and self.device.index is None:
            # pin the index: engine threads (AsyncEngine, kvx) start on device 0
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.is_gpu = self.device.type == "cuda"
        self.tp_size = get_state().tp_size
        if self.is_gpu:
            from llmd_amd.ops.gemm_tuning import enable_lookup

            tuned = enable_lookup()
            if tuned:
                log.info("GEMM selection from %s", tuned)
        self.bs = cfg.cache.block_size
        self.max_model_len = cfg.sched.max_model_len
        self.width = math.ceil(self.max_model_len / self.bs) + 1
        torch.manual_seed(cfg.seed)
        t0 = time.time()
        from llmd_amd.parallel import eplb

        eplb.configure(cfg.parallel.enable_eplb, cfg.parallel.eplb_config)
        self.model = build_model(self.mc, device=self.device, max_pos=self.max_model_len + 1)
        if cfg.load_format in ("safetensors", "auto") and cfg.weights_path:
            from llmd_amd.models.loader import load_weights

            load_weights(self.model, cfg.weights_path)
        if cfg.quantization == "fp8":
            from llmd_amd.models.layers import quantize_fp8

            n = quantize_fp8(self.model)
            log.info("fp8 W8A8: quantised %d linears", n)
        elif cfg.quantization == "mxfp4":
            from llmd_amd.models.layers import quantize_mxfp4

            n = quantize_mxfp4(self.model)
            log.info("mxfp4 experts + fp8 W8A8 linears: quantised %d tensors", n)
        elif cfg.quantization:
            raise ValueError(f"unsupported quantization {cfg.quantization}")
        if self.is_gpu:
            torch.cuda.synchronize()
        log.info("model %s built in %.1fs", self.mc.name, time.time() - t0)
        attn = self.model.attention_layers()
        self.Hkv, self.D, self.L = attn[0].Hkv, attn[0].D, len(attn)
        self.Hq = attn[0].Hq
        # cache geometry per layer: (planes, heads, dim) - K/V planes of GQA heads,
        # or one latent row per token for MLA
        self.kv_spec = self.model.kv_spec() if hasattr(self.model, "kv_spec") else (2, self.Hkv, self.D)
        self.is_mla = bool(getattr(self.model, "needs_mla_rows", False))
        # KV storage dtype (vLLM --kv-cache-dtype): bf16 or OCP fp8
        # e4m3fn (gfx950 native) with per-layer dequant scales (k_scale/v_scale,
        # 1.0 unless the checkpoint carries calibrated ones).
        kvd = (cfg.cache.kv_cache_dtype or "auto").lower()
        if kvd in ("auto", "bf16", "bfloat16"):
            self.kv_dtype = torch.bfloat16
        elif kvd in ("fp8", "fp8_e4m3", "fp8_e4m3fn"):
            self.kv_dtype = torch.float8_e4m3fn
        else:
            raise ValueError(f"unsupported --kv-cache-dtype {cfg.cache.kv_cache_dtype}")
        # shared-prefix decode (ops.shared_prefix_plan): GQA kernels only; sliding-window
        # layers (gpt-oss) keep the plain kernel, so the step's split must also cover
        # their window (self.max_window)
        G = self.Hq // self.Hkv
        self.max_window = max((a.window for a in attn if a.window), default=0)
        self.cascade_ok = (cfg.cache.shared_prefix_decode and cfg.cache.enable_prefix_caching and not self.is_mla
                           and G <= 16 and 16 % G == 0)
        self.casc_variant = ops.cascade_variant(G, self.D, self.bs, self.kv_dtype != torch.bfloat16)
        self.cascade_ok = self.cascade_ok and self.casc_variant is not None
        self.casc_work = max(16, -(-512 // self.Hkv))  # prefix work units: ~2 workgroups per CU over kv heads
        self.casc_slots = 16                           # prefix partial slots per sequence
        self.cgraphs: dict[int, tuple] = {}
        self.lora = None  # engine/lora.py LoRAManager (set by the engine / TP follower)
        self.kv = None
        self.num_blocks = 0
        # hybrid KV cache: windowed layers in their own pool (engine/hybrid_kv.py)
        self.swa_layers = [i for i, a in enumerate(attn) if getattr(a, "window", 0)]
        self.full_layers = [i for i in range(self.L) if i not in set(self.swa_layers)]
        self.hybrid = self._want_hybrid()
        self.kv_swa = None
        self.num_swa_blocks = 0
        if self.hybrid:
            log.info("hybrid KV cache: %d full-attention layers, %d window-%d layers in their own pool",
                     len(self.full_layers), len(self.swa_layers), self.max_window)
        self.graphs: dict[int, tuple] = {}
        self.dbo_graphs: dict[int, tuple] = {}  # bucket -> (graph, logits) of two B/2 micro-batches
        self._rng = np.random.default_rng(cfg.seed)
        self.graph_plans: dict[int, tuple] = {}
        self._init_symm()

    def eplb_tick(self):
        """Count one executed forward for EPLB; rebalances every step_interval."""
        from llmd_amd.parallel import eplb

        if not eplb.config().enabled:
            return False
        mods = [m for m in self.model.modules() if getattr(m, "eplb", None) is not None]
        return eplb.on_forward(group=get_state().ep_group,
                               params_of=lambda: [(m.eplb, m.expert_params()) for m in mods])

    def _init_symm(self):
        """Symmetric IPC heap users (parallel/symm.py): the TP custom all-reduce
        and the wide-EP low-latency dispatch/combine. Collective: every rank of
        the group constructs its runner, so the handle exchange lines up."""
        if not self.is_gpu:
            return
        from llmd_amd.parallel import ep as ep_mod
        from llmd_amd.parallel import symm

        st = get_state()
        pc = self.cfg.parallel
        if self.tp_size > 1:
            from llmd_amd.parallel.comm import warm_tp_group

            warm_tp_group(self.device)
        if self.tp_size > 1 and not pc.disable_custom_all_reduce and symm.enabled_by_env():
            # every TP rank must agree: a rank that could not map a peer's heap
            # would otherwise wait on epochs its peers never write
            ok = 1
            try:
                symm.init(st.tp_rank, st.tp_size, group=st.tp_cpu_group, tp_allreduce=True)
            except Exception as e:  # noqa: BLE001 - fall back to RCCL all-reduce
                log.warning("custom all-reduce unavailable (%s); using RCCL", e)
                ok = 0
            from llmd_amd.parallel.comm import tp_min_int

            if tp_min_int(ok) == 0:
                symm.shutdown()
        elif (ep_mod.canonical(pc.all2all_backend) in ("symm_ll", "symm_ht") and st.dp_size > 1
              and st.tp_size == 1 and self.mc.is_moe):
            # LL: decode-sized steps in one exchange; HT: prefill steps in chunks of this many rows
            rows = max(self.cfg.cuda_graph_max_bs, 256)
            if ep_mod.canonical(pc.all2all_backend) == "symm_ht":
                rows = max(rows, int(os.environ.get("LLMD_EP_HT_ROWS", "1024")))
            # block-fp8 experts: quantise in the dispatch kernel (DeepEP-LL use_fp8)
            fp8 = (os.environ.get("LLMD_EP_FP8_DISPATCH", "1") == "1"
                   and any(getattr(m, "w1_scale", None) is not None
                           and m.w1.dtype in (torch.float8_e4m3fn, torch.uint8)
                           for m in self.model.modules()))
            symm.init(st.ep_rank, st.ep_size, group=st.cpu_group, ep_rows=rows, hidden=self.mc.hidden_size,
                      topk=self.mc.num_experts_per_tok, micro_batches=2 if pc.enable_dbo else 1, ep_fp8=fp8)

    # ------------------------------------------------------------ KV cache
    def _want_hybrid(self) -> bool:
        """Hybrid manager: on by default for models mixing windowed and full layers
        (vLLM's default); off with --disable-hybrid-kv-cache-manager. kvx P/D and the
        tiered offload move / store both pools."""
        flag = self.cfg.cache.hybrid_kv_cache_manager
        if not self.swa_layers or not self.full_layers or self.is_mla or flag is False:
            return False
        if self.cfg.parallel.enable_dbo:
            return False  # dual-batch graphs carry one set of tables
        return True

    def layer_bytes_per_block(self) -> int:
        planes, heads, dim = self.kv_spec
        return planes * heads * self.bs * dim * torch.empty(0, dtype=self.kv_dtype).element_size()

    def block_bytes(self) -> int:
        """Bytes of one block of the main pool (all layers, or the full-attention
        layers of a hybrid cache)."""
        n = len(self.full_layers) if self.hybrid else self.L
        return n * self.layer_bytes_per_block()

    def swa_block_bytes(self) -> int:
        return len(self.swa_layers) * self.layer_bytes_per_block()

    def _swa_pool_blocks(self) -> int:
        from .hybrid_kv import swa_blocks

        sc = self.cfg.sched
        return swa_blocks(sc.max_num_seqs, sc.max_num_batched_tokens, self.max_window, self.bs)

    def _wants_vmm(self) -> bool:
        """KV producers export their pool to other processes (kvx); a single
        >4 GiB allocation cannot be imported through hipIpc on this stack, so
        the pool is built from exportable 2 GiB VMM chunks (kvx_vmm.hip)."""
        kt = self.cfg.kv_transfer_config or {}
        return (self.is_gpu and kt.get("kv_role") in ("kv_producer", "kv_both")
                and os.environ.get("LLMD_KV_VMM", "1") != "0")

    def _alloc_cache(self, num_blocks: int, scratch: bool = False) -> torch.Tensor:
        planes, heads, dim = self.kv_spec
        shape = (len(self.full_layers) if self.hybrid else self.L, num_blocks, planes, heads, self.bs, dim)
        if self.hybrid:
            self.kv_swa = torch.zeros((len(self.swa_layers), num_blocks if scratch else self.num_swa_blocks,
                                       planes, heads, self.bs, dim), dtype=self.kv_dtype, device=self.device)
        self.vmm = None
        if not scratch and self._wants_vmm():
            C = ops.native()
            chunk = VMM_CHUNK
            gran = C.vmm_granularity(self.device.index)
            chunk = (chunk + gran - 1) // gran * gran
            need = num_blocks * self.block_bytes()
            n = (need + chunk - 1) // chunk
            pool, fds = C.vmm_pool(self.device.index, chunk, n)
            kv = pool[:need].view(self.kv_dtype).view(shape)
            self.vmm = {"fds": list(fds), "chunk": chunk, "n": n, "pool": pool}
        else:
            kv = torch.empty(shape, dtype=self.kv_dtype, device=self.device)
        self._bind(kv)
        return kv

    def _bind(self, kv: Optional[torch.Tensor]):
        if kv is None:
            self.kv_swa = None
        slot = {}
        if self.hybrid:
            slot.update({li: ("full", j) for j, li in enumerate(self.full_layers)})
            slot.update({li: ("swa", j) for j, li in enumerate(self.swa_layers)})
        for i, a in enumerate(self.model.attention_layers()):
            pool, j = slot.get(i, ("full", i))
            src = kv if pool == "full" else self.kv_swa
            if hasattr(a, "bind_cache"):
                a.bind_cache(src[j]) if src is not None else setattr(a, "cache", None)
            else:
                a.k_cache = src[j, :, 0] if src is not None else None
                a.v_cache = src[j, :, 1] if src is not None else None

    def _mla_rows(self, meta: AttnMeta, nd: int, p_ql, p_ctx):
        """Row metadata of the latent-attention kernel (decode rows + one row per
        prefill token with its causal key count)."""
        dev = self.device
        if nd:
            meta.mla_d_rows = torch.arange(nd, dtype=torch.int32).to(dev, non_blocking=True)
        if p_ql:
            ql = np.asarray(p_ql, dtype=np.int64)
            ctx = np.asarray(p_ctx, dtype=np.int64)
            seq = np.repeat(np.arange(len(ql), dtype=np.int32), ql)
            first = np.repeat(ctx - ql, ql)
            within = np.arange(int(ql.sum()), dtype=np.int64) - np.repeat(np.cumsum(ql) - ql, ql)
            meta.p_row_seq = torch.from_numpy(seq).to(dev, non_blocking=True)
            meta.p_row_len = torch.from_numpy((first + within + 1).astype(np.int32)).to(dev, non_blocking=True)
            meta.p_max_ctx = int(ctx.max())

    @torch.no_grad()
    def profile_and_allocate(self) -> int:
        cc = self.cfg.cache
        if cc.num_gpu_blocks:
            nb = cc.num_gpu_blocks
        elif not self.is_gpu:
            budget = cc.kv_cache_memory_bytes or (256 << 20)
            if self.hybrid:
                budget -= self._swa_pool_blocks() * self.swa_block_bytes()
            nb = max(64, budget // self.block_bytes())
        else:
            # dummy max-size step on a scratch cache to measure activation peak
            T = self.cfg.sched.max_num_batched_tokens
            scratch_blocks = math.ceil(T / self.bs) + 2
            self.kv = self._alloc_cache(scratch_blocks, scratch=True)
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            self._dummy_prefill(T, scratch_blocks)
            torch.cuda.synchronize()
            act_peak = torch.cuda.max_memory_allocated() - base
            self.kv = None
            self._bind(None)
            torch.cuda.empty_cache()
            free, total = torch.cuda.mem_get_info()
            if cc.kv_cache_memory_bytes:
                budget = cc.kv_cache_memory_bytes
            else:
                used = total - free
                budget = int(total * cc.gpu_memory_utilization) - used - act_peak - (2 << 30)
            if self.hybrid:  # the windowed pool first, the full-attention layers get the rest
                self.num_swa_blocks = self._swa_pool_blocks()
                budget -= self.num_swa_blocks * self.swa_block_bytes()
            nb = max(16, budget // self.block_bytes())
            log.info("kv cache: %d blocks x %d tokens (%.1f GiB), activation peak %.2f GiB",
                     nb, self.bs, nb * self.block_bytes() / 2**30, act_peak / 2**30)
        if self.tp_size > 1:
            nb = tp_min_int(int(nb))  # every TP rank must hold the same block pool
        self.num_blocks = int(nb)
        if self.hybrid:
            self.num_swa_blocks = self._swa_pool_blocks()
            log.info("hybrid KV cache: %d full-layer blocks (%d tokens of context) + %d windowed blocks",
                     self.num_blocks, self.num_blocks * self.bs, self.num_swa_blocks)
        self.kv = self._alloc_cache(self.num_blocks)
        return self.num_blocks

    def _dummy_prefill(self, T: int, nblocks: int):
        nseq = max(1, math.ceil(T / self.bs))
        ql = [min(self.bs, T - i * self.bs) for i in range(nseq)]
        ql = [q for q in ql if q > 0]
        bt = np.zeros((len(ql), self.width), dtype=np.int32)
        for i in range(len(ql)):
            bt[i, 0] = i % nblocks
        ids = torch.zeros(sum(ql), dtype=torch.long, device=self.device)
        pos = torch.cat([torch.arange(q) for q in ql]).to(self.device)
        slots = torch.cat([torch.arange(q) + (i % nblocks) * self.bs for i, q in enumerate(ql)]).to(self.device)
        qs = np.cumsum([0] + ql[:-1]).astype(np.int32)
        meta = AttnMeta(num_tokens=sum(ql), positions=pos, slot_mapping=slots,
                        num_prefill_tokens=sum(ql),
                        p_block_tables=torch.from_numpy(bt).to(self.device),
                        p_q_start=torch.from_numpy(qs).to(self.device),
                        p_q_len=torch.tensor(ql, dtype=torch.int32, device=self.device),
                        p_ctx_len=torch.tensor(ql, dtype=torch.int32, device=self.device))
        meta.p_items = self._items(ql, ql)
        if self.is_mla:
            self._mla_rows(meta, 0, ql, ql)
        h = self.model(ids, meta)
        self.model.compute_logits(h[: min(len(ql), self.cfg.sched.max_num_seqs)])

    def _items(self, q_len, ctx_len):
        tpi = ops.prefill_tokens_per_item(self.Hq, self.Hkv, self.D, self.cfg.cache.block_size,
                                          self.kv_dtype == torch.float8_e4m3fn)
        it = ops.build_prefill_items(list(q_len), list(ctx_len), tpi)
        return torch.tensor(it, dtype=torch.int32).view(-1, 2).to(self.device, non_blocking=True)

    # ------------------------------------------------------------ inputs
    def _prepare(self, so: SchedulerOutput, block_tables: dict[int, list[int]]):
        dec, pre = so.decodes, so.prefills
        nd = len(dec)
        ids, pos, slots = [], [], []
        bs = self.bs
        d_bt = np.zeros((nd, self.width), dtype=np.int32)
        d_len = np.zeros(nd, dtype=np.int32)
        for i, sr in enumerate(dec):
            r = sr.req
            p = sr.start
            tok = r.token_at(p)
            bt = block_tables[r.seq_id]
            ids.append(tok)
            pos.append(p)
            slots.append(bt[p // bs] * bs + p % bs)
            d_bt[i, : len(bt)] = bt
            d_len[i] = p + 1
        p_ql, p_ctx = [], []
        p_bt = np.zeros((len(pre), self.width), dtype=np.int32)
        for i, sr in enumerate(pre):
            r = sr.req
            bt = block_tables[r.seq_id]
            toks = r.token_range(sr.start, sr.start + sr.num_new_tokens)
            ids.extend(toks)
            ps = np.arange(sr.start, sr.start + sr.num_new_tokens)
            pos.extend(ps.tolist())
            bta = np.asarray(bt, dtype=np.int64)
            slots.extend((bta[ps // bs] * bs + ps % bs).tolist())
            p_bt[i, : len(bt)] = bt
            p_ql.append(sr.num_new_tokens)
            p_ctx.append(sr.start + sr.num_new_tokens)
        return ids, pos, slots, d_bt, d_len, p_ql, p_ctx, p_bt

    def _group_tables(self, so: SchedulerOutput, tables: dict):
        """Slot mapping and block tables of one KV group (the windowed pool of a
        hybrid cache): same token layout as _prepare."""
        bs = self.bs
        slots = []
        d_bt = np.zeros((len(so.decodes), self.width), dtype=np.int32)
        for i, sr in enumerate(so.decodes):
            bt = tables[sr.req.seq_id]
            p = sr.start
            slots.append(bt[p // bs] * bs + p % bs)
            d_bt[i, : len(bt)] = bt
        p_bt = np.zeros((len(so.prefills), self.width), dtype=np.int32)
        for i, sr in enumerate(so.prefills):
            bt = tables[sr.req.seq_id]
            ps = np.arange(sr.start, sr.start + sr.num_new_tokens)
            bta = np.asarray(bt, dtype=np.int64)
            slots.extend((bta[ps // bs] * bs + ps % bs).tolist())
            p_bt[i, : len(bt)] = bt
        return slots, d_bt, p_bt

    def _sample_rows(self, so: SchedulerOutput):
        """Rows (token index) that produce a sampled token, and their requests."""
        rows, reqs = [], []
        for i, sr in enumerate(so.decodes):
            if sr.samples:
                rows.append(i)
                reqs.append(sr.req)
        off = len(so.decodes)
        for sr in so.prefills:
            off += sr.num_new_tokens
            if sr.samples:
                rows.append(off - 1)
                reqs.append(sr.req)
        return rows, reqs

    def _sampling_tensors(self, reqs):
        n = len(reqs)
        temps = np.zeros(n, dtype=np.float32)
        seeds = np.zeros(n, dtype=np.int64)
        topk = np.zeros(n, dtype=np.int32)
        topp = np.ones(n, dtype=np.float32)
        any_rand = any_k = any_p = False
        for i, r in enumerate(reqs):
            sp = r.params
            if sp.temperature > 0:
                any_rand = True
                temps[i] = sp.temperature
                base = sp.seed if sp.seed is not None else r.extra.setdefault(
                    "_seed", int(self._rng.integers(0, 2**62)))
                seeds[i] = _mix64(base * 1000003 + len(r.output_token_ids))
            if sp.top_k > 0:
                topk[i] = sp.top_k
                any_k = True
            if sp.top_p < 1.0:
                topp[i] = sp.top_p
                any_p = True
        return temps, seeds, topk, topp, any_rand, any_k, any_p

    # ------------------------------------------------------------ execution
    @torch.no_grad()
    def execute(self, so: SchedulerOutput, block_tables: dict[int, list[int]], force_eager: bool = False,
                bucket: Optional[int] = None, prev: Optional["DeferredSample"] = None, defer: bool = False):
        """force_eager / bucket: DP-lockstep overrides (every EP rank must run the
        same kind of step with the same collective shapes).

        Async scheduling (engine.py): ``prev`` is the previous step, still in flight, whose
        sampled tokens are the inputs of this step's decode rows - they are gathered on the
        device (the host holds placeholders); ``defer`` returns a DeferredSample instead of
        waiting for this step's tokens."""
        if so.empty:
            return DeferredSample.empty() if defer else {}
        with markers.range("llmd.plan"):
            pl, reqs = self.plan(so, block_tables)
            if force_eager:
                pl["graph"] = False
            elif bucket is not None and pl["graph"]:
                pl["bucket"] = bucket
            if prev is not None:
                g = self._gather_from(so, prev)
                if g is not None:
                    pl["gather"] = g
            if self.tp_size > 1:
                assert "gather" not in pl, "async scheduling is single-rank only"
                tp_broadcast_plan(pl)  # TP followers run the same plan (engine/tp_worker.py)
        with markers.range("llmd.forward"):
            logits = self.run_plan(pl)
        if not reqs:
            return DeferredSample.empty() if defer else {}
        if pl.get("embed") and getattr(self, "_last_hidden", None) is not None:
            # pooling for /v1/embeddings: last-token final hidden state, L2-normalised
            e = torch.nn.functional.normalize(self._last_hidden.float(), dim=-1).cpu()
            for i, r in enumerate(reqs):
                if r.params.embed:
                    r.extra["embedding"] = e[i].tolist()
        with markers.range("llmd.sample"):
            ids, lp = self._sample_dev(logits, reqs)
            if defer:
                return DeferredSample(ids, lp, [r.seq_id for r in reqs], self.is_gpu)
            return self._to_host(ids, lp, reqs)

    def _gather_from(self, so: SchedulerOutput, prev: "DeferredSample"):
        """(dst rows, src rows) device index tensors: decode rows whose input token is the
        previous step's sampled token (a host placeholder), or None."""
        dst, src = [], []
        for i, sr in enumerate(so.decodes):
            r = sr.req
            if r.async_pending and sr.start == r.num_tokens - 1:
                dst.append(i)
                src.append(prev.row_of[r.seq_id])
        if not dst:
            return None
        return (torch.tensor(dst, dtype=torch.long).to(self.device, non_blocking=True),
                torch.tensor(src, dtype=torch.long).to(self.device, non_blocking=True), prev.ids)

    def plan(self, so: SchedulerOutput, block_tables: dict[int, list[int]]) -> tuple[dict, list]:
        """Host-side step description: everything a (TP) rank needs to run the
        forward, independent of the scheduler's request objects."""
        rows, reqs = self._sample_rows(so)
        ids, pos, slots, d_bt, d_len, p_ql, p_ctx, p_bt = self._prepare(so, block_tables)
        graph = not so.prefills and self._graph_ok(len(so.decodes))
        pl = {"graph": graph, "nd": len(so.decodes), "ids": ids, "pos": pos, "slots": slots, "d_bt": d_bt,
              "d_len": d_len, "p_ql": p_ql, "p_ctx": p_ctx, "p_bt": p_bt, "rows": rows}
        if self.hybrid:
            pl["swa"] = self._group_tables(so, block_tables.swa)
        if self.lora is not None:
            lo = [sr.req.lora_id for sr in so.decodes]
            for sr in so.prefills:
                lo.extend([sr.req.lora_id] * sr.num_new_tokens)
            pl["lora"] = lo
        mm = self._mm_rows(so)
        if mm is not None:
            pl["mm"] = mm
        if any(r.params.embed for r in reqs):
            pl["embed"] = True
            pl["graph"] = False
        return pl, reqs

    def _mm_rows(self, so: SchedulerOutput):
        """Image-placeholder rows of this step's prefill chunks + their embeddings."""
        if not any(sr.req.mm_inputs for sr in so.prefills):
            return None
        from llmd_amd.models.vision import chunk_mm_rows

        rows, embs = [], []
        row0 = len(so.decodes)
        for sr in so.prefills:
            if sr.req.mm_inputs:
                r, e = chunk_mm_rows(sr.req.mm_inputs, sr.start, sr.num_new_tokens, row0)
                rows += r
                embs += e
            row0 += sr.num_new_tokens
        if not rows:
            return None
        return rows, torch.cat([e.to(self.device) for e in embs])

    @torch.no_grad()
    def run_plan(self, pl: dict):
        # rccl kvx transport: KV sends / recvs are enqueued only between forward passes, so on every
        # rank the p2p communicator's operations and this step's TP / EP collectives are issued in
        # one fixed order (kvx/agent.py p2p_step_guard; a no-op without the rccl transport)
        with p2p_step_guard():
            return self._run_plan(pl)

    def _run_plan(self, pl: dict):
        rows = pl["rows"]
        if self.lora is not None:
            lo = pl.get("lora") or [0] * len(pl["ids"])
            if pl["graph"]:  # padded rows of the bucket must not pick up stale adapter slots
                lo = list(lo) + [0] * ((pl.get("bucket") or self._bucket(pl["nd"])) - len(lo))
            self.lora.set_tokens(lo)
        if pl["graph"]:
            return self._run_decode_graph(pl)
        h = self._run_eager(pl)
        if not rows:
            return None
        idx = torch.tensor(rows, dtype=torch.long).to(self.device, non_blocking=True)
        hs = h.index_select(0, idx)
        self._last_hidden = hs if pl.get("embed") else None
        return self.model.compute_logits(hs)

    def _penalize(self, logits, reqs):
        """Presence / frequency / repetition penalties, logit bias and min-p for
        the rows whose requests ask for them (one scatter per kind; rows
        without them are untouched, so ordinary steps pay nothing)."""
        logits = logits.float()
        dev = logits.device
        pr, pt, pv, rr, rt, rv = [], [], [], [], [], []
        mp_rows, mp_vals, mp_temps = [], [], []
        for i, r in enumerate(reqs):
            sp = r.params
            if not sp.penalized:
                continue
            out = np.asarray(r.output_token_ids, dtype=np.int64)
            if (sp.presence_penalty or sp.frequency_penalty) and out.size:
                toks, cnt = np.unique(out, return_counts=True)
                pr.append(np.full(toks.size, i))
                pt.append(toks)
                pv.append(sp.frequency_penalty * cnt + sp.presence_penalty)
            if sp.logit_bias:
                toks = np.fromiter(sp.logit_bias.keys(), dtype=np.int64)
                pr.append(np.full(toks.size, i))
                pt.append(toks)
                pv.append(-np.fromiter(sp.logit_bias.values(), dtype=np.float64))
            if sp.repetition_penalty != 1.0:
                seen = np.unique(np.concatenate([np.asarray(r.prompt_token_ids, dtype=np.int64), out]))
                rr.append(np.full(seen.size, i))
                rt.append(seen)
                rv.append(np.full(seen.size, sp.repetition_penalty))
            if sp.min_p > 0.0:
                mp_rows.append(i)
                mp_vals.append(sp.min_p)
                mp_temps.append(max(sp.temperature, 1e-5))
        if rr:
            ri = torch.from_numpy(np.concatenate(rr)).to(dev)
            ti = torch.from_numpy(np.concatenate(rt)).to(dev)
            rp = torch.from_numpy(np.concatenate(rv)).to(dev, torch.float32)
            cur = logits[ri, ti]
            logits[ri, ti] = torch.where(cur > 0, cur / rp, cur * rp)
        if pr:
            ri = torch.from_numpy(np.concatenate(pr)).to(dev)
            ti = torch.from_numpy(np.concatenate(pt)).to(dev)
            logits.index_put_((ri, ti), -torch.from_numpy(np.concatenate(pv)).to(dev, torch.float32),
                              accumulate=True)
        if mp_rows:
            rows = torch.tensor(mp_rows, device=dev)
            sub = logits.index_select(0, rows) / torch.tensor(mp_temps, device=dev).unsqueeze(1)
            pr_ = torch.softmax(sub, dim=-1)
            thr = pr_.max(dim=-1, keepdim=True).values * torch.tensor(mp_vals, device=dev).unsqueeze(1)
            keep = logits.index_select(0, rows).masked_fill(pr_ < thr, float("-inf"))
            logits.index_copy_(0, rows, keep)
        return logits

    def _sample(self, logits, reqs):
        ids, lp = self._sample_dev(logits, reqs)
        return self._to_host(ids, lp, reqs)

    @staticmethod
    def _to_host(ids, lp, reqs):
        ids_h = ids.cpu().tolist()
        lp_h = lp.cpu().tolist() if lp is not None else [0.0] * len(ids_h)
        return {r.seq_id: (int(ids_h[i]), float(lp_h[i])) for i, r in enumerate(reqs)}

    def _sample_dev(self, logits, reqs):
        temps, seeds, topk, topp, any_rand, any_k, any_p = self._sampling_tensors(reqs)
        want_lp = any(r.params.logprobs for r in reqs)
        dev = self.device
        if any(r.params.penalized for r in reqs):
            logits = self._penalize(logits, reqs)
        if any_k or any_p:
            logits = logits.float()
            ops.topk_topp_mask(logits, torch.from_numpy(topk).to(dev) if any_k else None,
                               torch.from_numpy(topp).to(dev) if any_p else None,
                               torch.from_numpy(temps).to(dev))
        t = torch.from_numpy(temps).to(dev, non_blocking=True) if any_rand else None
        s = torch.from_numpy(seeds).to(dev, non_blocking=True) if any_rand else None
        gen = None
        if not self.is_gpu and any_rand:
            gen = torch.Generator().manual_seed(int(seeds[0]) & 0x7FFFFFFF)
        return ops.sample(logits, t, s, want_logprob=want_lp, generator=gen)

    def _run_eager(self, pl: dict):
        ids, meta = self._eager_meta(pl)
        return self.model(ids, meta)

    def _eager_meta(self, pl: dict):
        ids, pos, slots, d_bt, d_len = pl["ids"], pl["pos"], pl["slots"], pl["d_bt"], pl["d_len"]
        p_ql, p_ctx, p_bt = pl["p_ql"], pl["p_ctx"], pl["p_bt"]
        dev = self.device
        nd = pl["nd"]
        T = len(ids)
        swa = pl.get("swa")
        host = torch.tensor([ids, pos, slots] + ([swa[0]] if swa is not None else []), dtype=torch.long)
        if self.is_gpu:
            host = host.pin_memory()
        hd = host.to(dev, non_blocking=True)
        meta = AttnMeta(num_tokens=T, positions=hd[1], slot_mapping=hd[2], num_decode=nd)
        if nd:
            meta.d_block_tables = torch.from_numpy(d_bt).to(dev, non_blocking=True)
            meta.d_seq_lens = torch.from_numpy(d_len).to(dev, non_blocking=True)
            meta.d_max_ctx = int(d_len.max())
            mctx = meta.d_max_ctx
            plan = self._cascade_plan(d_bt, d_len)
            if plan is not None:
                meta.d_cascade = ops.cascade_tensors(plan, dev)
                # splits cover the longest own suffix (and a windowed layer's window)
                mctx = max(int((d_len - plan.sstart[:nd]).max()), min(self.max_window, mctx))
            meta.d_split = ops.decode_split_plan(mctx, nd, self.Hkv, self.Hq // self.Hkv)
        if p_ql:
            meta.num_prefill_tokens = sum(p_ql)
            meta.p_block_tables = torch.from_numpy(p_bt).to(dev, non_blocking=True)
            qs = np.cumsum([0] + p_ql[:-1]).astype(np.int32)
            meta.p_q_start = torch.from_numpy(qs).to(dev, non_blocking=True)
            meta.p_q_len = torch.tensor(p_ql, dtype=torch.int32).to(dev, non_blocking=True)
            meta.p_ctx_len = torch.tensor(p_ctx, dtype=torch.int32).to(dev, non_blocking=True)
            meta.p_items = self._items(p_ql, p_ctx)
        if self.is_mla:
            self._mla_rows(meta, nd, p_ql, p_ctx)
        if pl.get("mm") is not None:
            rows, embs = pl["mm"]
            meta.mm_rows = torch.tensor(rows, dtype=torch.long).to(dev, non_blocking=True)
            meta.mm_embeds = embs.to(dev)
        if swa is not None:  # windowed layers: their own pool's slots and block tables
            meta.swa = dataclasses.replace(
                meta, slot_mapping=hd[3], d_cascade=None,
                d_block_tables=torch.from_numpy(swa[1]).to(dev, non_blocking=True) if nd else None,
                p_block_tables=torch.from_numpy(swa[2]).to(dev, non_blocking=True) if p_ql else None)
        ids = hd[0]
        if pl.get("gather") is not None:  # async: decode inputs sampled by the step still in flight
            dst, src, prev_ids = pl["gather"]
            ids.index_copy_(0, dst, prev_ids.index_select(0, src).to(ids.dtype))
        return ids, meta

    def _cascade_plan(self, d_bt, d_len, max_work=None):
        """Shared-prefix decode plan for this step's decode rows, or None."""
        if not self.cascade_ok or len(d_len) < 2:
            return None
        return ops.shared_prefix_plan(d_bt, d_len, self.bs, self.Hq // self.Hkv, self.Hkv,
                                      variant=self.casc_variant, max_slots=self.casc_slots, max_work=max_work)

    # ------------------------------------------------------------ dual-batch overlap
    def _forward_steps(self, ids, meta):
        """model.forward as a generator yielding after every decoder layer
        (embed -> layers -> norm is the structure of every model here)."""
        m = self.model
        x = m.embed(ids)
        residual = None
        for layer in m.layers:
            x, residual = layer(x, residual, meta)
            yield None
        x, _ = m.norm(x, residual)
        yield x

    @torch.no_grad()
    def execute_dbo(self, so: Optional[SchedulerOutput], block_tables: dict, bucket: Optional[int] = None) -> dict:
        """Dual-batch overlap (reference --enable-dbo,
        guides/wide-ep-lws/modelserver/gpu/vllm/base/decode.yaml:112-113,
        prefill.yaml:83-84) for a wide-EP step: the step splits into two micro-batches,
        each with its own attention metadata and its own symm EP channel /
        receive buffers; their layers are issued alternately on two HIP
        streams so one micro-batch's dispatch/combine kernels (bounded to 64
        workgroups) run while the other's attention/expert GEMMs occupy the
        remaining CUs. ``so=None``: idle DP rank, two one-token dummy halves.
        ``bucket``: replay the captured dual-batch graph of that size instead
        (the caller sets the EP step rows to bucket/2 on every rank)."""
        from llmd_amd.parallel import symm

        if bucket is not None and (so is None or not any(sr.req.params.embed for sr in so.decodes)):
            return self._replay_dbo(so, block_tables, bucket)
        plans, reqs = [], []
        if so is None or so.empty:
            for _ in range(2):
                w = self.width
                plans.append({"graph": False, "nd": 1, "ids": [0], "pos": [0], "slots": [-1],
                              "d_bt": np.zeros((1, w), np.int32), "d_len": np.ones(1, dtype=np.int32),
                              "p_ql": [], "p_ctx": [], "p_bt": np.zeros((0, w), np.int32), "rows": []})
        else:
            for sub in self._dbo_split(so):
                if not sub.empty:
                    pl, rq = self.plan(sub, block_tables)
                else:  # odd split of a 1-token step: a dummy half keeps the collectives paired
                    w = self.width
                    pl, rq = ({"graph": False, "nd": 1, "ids": [0], "pos": [0], "slots": [-1],
                               "d_bt": np.zeros((1, w), np.int32), "d_len": np.ones(1, dtype=np.int32),
                               "p_ql": [], "p_ctx": [], "p_bt": np.zeros((0, w), np.int32), "rows": []}, [])
                plans.append(pl)
                reqs.append(rq)
        metas = [self._eager_meta(pl) for pl in plans]
        if self.is_gpu:
            main = torch.cuda.current_stream()
            if not hasattr(self, "_dbo_streams"):
                self._dbo_streams = (torch.cuda.Stream(device=self.device), torch.cuda.Stream(device=self.device))
            streams = self._dbo_streams
            for s in streams:
                s.wait_stream(main)
        gens = [self._forward_steps(ids, meta) for ids, meta in metas]
        outs = [None, None]
        done = [False, False]
        while not all(done):
            for m in (0, 1):
                if done[m]:
                    continue
                symm.set_active_mb(m)
                if self.is_gpu:
                    with torch.cuda.stream(streams[m]):
                        y = next(gens[m])
                else:
                    y = next(gens[m])
                if y is not None:
                    outs[m] = y
                    done[m] = True
        symm.set_active_mb(0)
        if self.is_gpu:
            for s in streams:
                main.wait_stream(s)
            for o in outs:
                o.record_stream(main)
        if so is None or so.empty:
            return {}
        logits, all_reqs = [], []
        for pl, rq, h in zip(plans, reqs, outs):
            if pl["rows"]:
                idx = torch.tensor(pl["rows"], dtype=torch.long).to(self.device, non_blocking=True)
                logits.append(self.model.compute_logits(h.index_select(0, idx)))
                all_reqs.extend(rq)
        if not all_reqs:
            return {}
        return self._sample(torch.cat(logits), all_reqs)

    @staticmethod
    def _dbo_split(so: SchedulerOutput) -> tuple[SchedulerOutput, SchedulerOutput]:
        """Two micro-batches of a step: decodes halved, then each prefill chunk
        to the half with fewer tokens so far (chunks are not split)."""
        h = (len(so.decodes) + 1) // 2
        halves = (SchedulerOutput(decodes=list(so.decodes[:h])), SchedulerOutput(decodes=list(so.decodes[h:])))
        for sr in sorted(so.prefills, key=lambda s: -s.num_new_tokens):
            min(halves, key=lambda x: x.num_tokens).prefills.append(sr)
        return halves

    # ------------------------------------------------------------ graphs
    def _bucket(self, n: int) -> int:
        b = 1
        while b < n:
            b *= 2
        return b

    def _graph_ok(self, n: int) -> bool:
        return self.is_gpu and not self.cfg.enforce_eager and bool(self.graphs) and \
            self._bucket(n) in self.graphs

    @torch.no_grad()
    def capture_graphs(self):
        if not self.is_gpu or self.cfg.enforce_eager:
            return
        maxb = min(self.cfg.cuda_graph_max_bs, self.cfg.sched.max_num_seqs)
        buckets = []
        b = 1
        while b <= maxb:
            buckets.append(b)
            b *= 2
        if buckets[-1] < maxb:
            buckets.append(self._bucket(maxb))
        M = buckets[-1]
        dev = self.device
        # per-bucket split plans (valid up to max_model_len): large buckets get few
        # long splits, small ones many - one fixed plan for all buckets starved the
        # big batches (2.6 TB/s KV read at batch 64 vs 4.7 with a sized plan)
        self.graph_plans = {B: ops.decode_split_plan(self.max_model_len, B, self.Hkv, self.Hq // self.Hkv)
                            for B in buckets}
        extra = self.casc_slots if self.cascade_ok else 0
        ws_rows = max(B * (p[1] + extra) for B, p in self.graph_plans.items())
        # shared-prefix decode inputs [sstart | pcount | members | work] (ops.cascade_tensors)
        self.g_casc = torch.zeros(3 * M + 5 * self.casc_work, dtype=torch.int32, device=dev)
        # keys per decode split, re-sized at every replay to the step's longest context (the
        # bucket's split count stays the grid): a plan sized for max_model_len would leave most
        # splits of a short-context batch empty and the chip underfilled
        self.g_split = torch.full((1,), self.graph_plans[buckets[-1]][0], dtype=torch.int32, device=dev)
        self.g_ids = torch.zeros(M, dtype=torch.long, device=dev)
        self.g_pos = torch.zeros(M, dtype=torch.long, device=dev)
        self.g_slots = torch.full((M,), -1, dtype=torch.long, device=dev)
        self.g_bt = torch.zeros(M, self.width, dtype=torch.int32, device=dev)
        self.g_len = torch.ones(M, dtype=torch.int32, device=dev)
        if self.hybrid:  # the windowed pool's slots / tables (block 0 = null block)
            self.g_slots_swa = torch.full((M,), -1, dtype=torch.long, device=dev)
            self.g_bt_swa = torch.zeros(M, self.width, dtype=torch.int32, device=dev)
        self.g_ws = (torch.empty(ws_rows * self.Hq * self.D, dtype=torch.float32, device=dev),
                     torch.empty(ws_rows * self.Hq * 2, dtype=torch.float32, device=dev))
        if self.is_mla:  # fixed per-bucket latent-attention split plans + one shared workspace
            self.g_rows = torch.arange(M, dtype=torch.int32, device=dev)
            f8 = self.kv_dtype == torch.float8_e4m3fn
            self.mla_plans = {B: ops.mla_split_plan(self.max_model_len, B, self.Hq, fp8=f8) for B in buckets}
            need = max(B * p[1] for B, p in self.mla_plans.items())
            self.g_mla_ws = (torch.empty(need * self.Hq * 512, dtype=torch.float32, device=dev),
                             torch.empty(need * self.Hq * 2, dtype=torch.float32, device=dev))
            self.g_mla_split = torch.full((1,), self.mla_plans[buckets[-1]][0], dtype=torch.int32, device=dev)
        pool = torch.cuda.graph_pool_handle()
        t0 = time.time()
        for B in reversed(buckets):
            self.g_split.fill_(self.graph_plans[B][0])  # warm-up / capture runs: the max_model_len plan
            meta = AttnMeta(num_tokens=B, positions=self.g_pos[:B], slot_mapping=self.g_slots[:B],
                            num_decode=B, d_block_tables=self.g_bt[:B], d_seq_lens=self.g_len[:B],
                            d_split=self.graph_plans[B], d_workspace=self.g_ws, d_max_ctx=self.max_model_len,
                            d_split_dev=self.g_split)
            if self.hybrid:
                meta.swa = dataclasses.replace(meta, slot_mapping=self.g_slots_swa[:B],
                                               d_block_tables=self.g_bt_swa[:B])
            if self.is_mla:
                meta.mla_d_rows, meta.mla_split, meta.mla_workspace = self.g_rows[:B], self.mla_plans[B], self.g_mla_ws
                self.g_mla_split.fill_(self.mla_plans[B][0])
                meta.mla_split_dev = self.g_mla_split
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    h = self.model(self.g_ids[:B], meta)
                    lg = self.model.compute_logits(h)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                h = self.model(self.g_ids[:B], meta)
                lg = self.model.compute_logits(h)
            self.graphs[B] = (g, lg)
            if self.cascade_ok and B >= 2:
                # variant with the shared-prefix kernel (all-padding work units while capturing)
                meta.d_cascade = (self.g_casc[:3 * B + 5 * self.casc_work], self.casc_variant, self.casc_slots)
                if self.hybrid:
                    meta.swa = dataclasses.replace(meta.swa, d_cascade=None)
                with torch.cuda.stream(s):
                    self.model(self.g_ids[:B], meta)
                torch.cuda.current_stream().wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    h = self.model(self.g_ids[:B], meta)
                    lg = self.model.compute_logits(h)
                self.cgraphs[B] = (g, lg)
        if self._dbo_graphable():
            self._capture_dbo_graphs(buckets, pool)
        torch.cuda.synchronize()
        log.info("captured %d decode graphs (+%d shared-prefix, +%d dual-batch) in %.1fs", len(buckets),
                 len(self.cgraphs), len(self.dbo_graphs), time.time() - t0)

    # ------------------------------------------------------------ dual-batch overlap under hipGraphs
    def _dbo_graphable(self) -> bool:
        from llmd_amd.parallel import symm

        return bool(self.cfg.parallel.enable_dbo) and self.lora is None and symm.micro_batches() >= 2

    def _dbo_meta(self, m: int, h: int, ws) -> AttnMeta:
        """Attention metadata of micro-batch m: rows [m*h, (m+1)*h) of the static
        buffers, its own split-KV workspace (the halves run concurrently)."""
        lo, hi = m * h, (m + 1) * h
        meta = AttnMeta(num_tokens=h, positions=self.g_pos[lo:hi], slot_mapping=self.g_slots[lo:hi], num_decode=h,
                        d_block_tables=self.g_bt[lo:hi], d_seq_lens=self.g_len[lo:hi], d_split=self.graph_plans[h],
                        d_workspace=ws[0], d_max_ctx=self.max_model_len)
        if self.is_mla:
            meta.mla_d_rows, meta.mla_split, meta.mla_workspace = self.g_rows[:h], self.mla_plans[h], ws[1]
        return meta

    def _dbo_forward(self, B: int, metas, streams):
        """Layers of the two micro-batches issued alternately on their own
        streams, forked from and joined back into the current stream (which is
        the capture stream under torch.cuda.graph, so both branches are
        recorded as parallel graph nodes)."""
        from llmd_amd.parallel import symm

        h = B // 2
        cur = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(cur)
        gens = [self._forward_steps(self.g_ids[m * h:(m + 1) * h], metas[m]) for m in (0, 1)]
        outs = [None, None]
        while outs[0] is None or outs[1] is None:
            for m in (0, 1):
                if outs[m] is None:
                    symm.set_active_mb(m)
                    with torch.cuda.stream(streams[m]):
                        outs[m] = next(gens[m])
        symm.set_active_mb(0)
        for s in streams:
            cur.wait_stream(s)
        return self.model.compute_logits(torch.cat(outs))

    def _capture_dbo_graphs(self, buckets, pool):
        """One graph per bucket B >= 2 holding both micro-batches of B/2 rows
        (symm EP channel / receive buffers per micro-batch, R = B/2 rows per
        rank). Every EP rank captures the same buckets in the same order."""
        dev = self.device
        ws0 = (self.g_ws, getattr(self, "g_mla_ws", None))
        ws1 = (tuple(torch.empty_like(t) for t in self.g_ws),
               tuple(torch.empty_like(t) for t in self.g_mla_ws) if self.is_mla else None)
        if not hasattr(self, "_dbo_streams"):
            self._dbo_streams = (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev))
        streams = self._dbo_streams
        for B in reversed([b for b in buckets if b >= 2]):
            h = B // 2
            metas = [self._dbo_meta(0, h, ws0), self._dbo_meta(1, h, ws1)]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._dbo_forward(B, metas, streams)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                lg = self._dbo_forward(B, metas, streams)
            self.dbo_graphs[B] = (g, lg)

    def dbo_bucket(self, t_max: int) -> Optional[int]:
        """Captured dual-batch bucket for a lockstep step of at most t_max decode rows per rank."""
        b = self._bucket(max(t_max, 2))
        return b if b in self.dbo_graphs else None

    def _replay_dbo(self, so: Optional[SchedulerOutput], block_tables: dict, B: int) -> dict:
        """The first ceil(nd/2) decodes fill micro-batch 0 from row 0, the rest
        micro-batch 1 from row B/2; other rows are padding (slot -1, len 1).
        ``so=None``: idle DP rank, all padding."""
        g, lg = self.dbo_graphs[B]
        h = B // 2
        ids = np.zeros(B, np.int64)
        pos = np.zeros(B, np.int64)
        slots = np.full(B, -1, np.int64)
        bt = np.zeros((B, self.width), np.int32)
        ln = np.ones(B, np.int32)
        reqs, grow = [], []
        if so is not None and not so.empty:
            pl, reqs = self.plan(so, block_tables)
            nd = pl["nd"]
            h0 = (nd + 1) // 2
            if h0 > h or nd - h0 > h:
                raise ValueError(f"dual-batch bucket {B} too small for {nd} decodes")
            perm = np.concatenate([np.arange(h0), h + np.arange(nd - h0)]).astype(np.int64)
            ids[perm], pos[perm], slots[perm] = pl["ids"], pl["pos"], pl["slots"]
            bt[perm], ln[perm] = pl["d_bt"], pl["d_len"]
            grow = perm[pl["rows"]].tolist()
        host = torch.from_numpy(np.stack([ids, pos, slots])).pin_memory()
        self.g_ids[:B].copy_(host[0], non_blocking=True)
        self.g_pos[:B].copy_(host[1], non_blocking=True)
        self.g_slots[:B].copy_(host[2], non_blocking=True)
        self.g_bt[:B].copy_(torch.from_numpy(bt).pin_memory(), non_blocking=True)
        self.g_len[:B].copy_(torch.from_numpy(ln).pin_memory(), non_blocking=True)
        g.replay()
        if not reqs:
            return {}
        return self._sample(lg[torch.tensor(grow, dtype=torch.long).to(self.device, non_blocking=True)], reqs)

    @torch.no_grad()
    def execute_dummy(self, graph_bucket: Optional[int] = None):
        """Idle DP rank in a lockstep step: run a forward with no real tokens so
        the MoE collectives of the busy ranks complete."""
        w = self.width
        empty = np.zeros((0, w), dtype=np.int32)
        if graph_bucket is not None and graph_bucket in self.graphs:
            pl = {"graph": True, "nd": 0, "bucket": graph_bucket, "ids": [], "pos": [], "slots": [], "d_bt": empty,
                  "d_len": np.zeros(0, dtype=np.int32), "p_ql": [], "p_ctx": [], "p_bt": empty, "rows": []}
        else:  # one padding decode token: no cache write (slot -1), one visible key
            pl = {"graph": False, "nd": 1, "ids": [0], "pos": [0], "slots": [-1], "d_bt": np.zeros((1, w), np.int32),
                  "d_len": np.ones(1, dtype=np.int32), "p_ql": [], "p_ctx": [], "p_bt": empty, "rows": []}
        if self.lora is not None:
            pl["lora"] = []
        self.run_plan(pl)

    def _run_decode_graph(self, pl: dict):
        n, rows = pl["nd"], pl["rows"]
        B = pl.get("bucket") or self._bucket(n)
        g, lg = self.graphs[B]
        ids, pos, slots, d_bt, d_len = pl["ids"], pl["pos"], pl["slots"], pl["d_bt"], pl["d_len"]
        if B > n:
            pad = B - n
            ids = ids + [0] * pad
            pos = pos + [0] * pad
            slots = slots + [-1] * pad
            d_bt = np.concatenate([d_bt, np.zeros((pad, self.width), dtype=np.int32)])
            d_len = np.concatenate([d_len, np.ones(pad, dtype=np.int32)])
        host = torch.tensor([ids, pos, slots], dtype=torch.long).pin_memory()
        self.g_ids[:B].copy_(host[0], non_blocking=True)
        if pl.get("gather") is not None:  # async: decode inputs sampled by the step still in flight
            dst, src, prev_ids = pl["gather"]
            self.g_ids.index_copy_(0, dst, prev_ids.index_select(0, src).to(self.g_ids.dtype))
        self.g_pos[:B].copy_(host[1], non_blocking=True)
        self.g_slots[:B].copy_(host[2], non_blocking=True)
        self.g_bt[:B].copy_(torch.from_numpy(d_bt).pin_memory(), non_blocking=True)
        self.g_len[:B].copy_(torch.from_numpy(d_len).pin_memory(), non_blocking=True)
        if self.hybrid:
            s_slots, s_bt, _ = pl.get("swa") or ([], np.zeros((0, self.width), np.int32), None)
            if B > n:
                s_slots = list(s_slots) + [-1] * (B - n)
                s_bt = np.concatenate([s_bt, np.zeros((B - n, self.width), dtype=np.int32)])
            self.g_slots_swa[:B].copy_(torch.tensor(s_slots, dtype=torch.long).pin_memory(), non_blocking=True)
            self.g_bt_swa[:B].copy_(torch.from_numpy(s_bt).pin_memory(), non_blocking=True)
        longest = int(d_len.max())
        if B in self.cgraphs:
            plan = self._cascade_plan(d_bt, d_len, max_work=self.casc_work)
            if plan is not None:
                ops.cascade_tensors(plan, self.device, out=self.g_casc)
                g, lg = self.cgraphs[B]
                # the per-sequence kernel covers suffixes only (windowed layers: their window)
                longest = max(int((d_len - plan.sstart).max()), min(self.max_window, longest))
        if self.is_mla:  # latent attention: >= 4 key tiles per split (a split re-reads its rows' 128-head Q)
            nsplit = self.mla_plans[B][1]
            split = max(256, -(-int(d_len.max()) // (64 * nsplit)) * 64)
            self.g_mla_split.copy_(torch.tensor([split], dtype=torch.int32).pin_memory(), non_blocking=True)
        else:  # the step's own split plan for its real rows, within the captured grid's splits
            split, _ = ops.decode_split_plan(longest, max(1, n), self.Hkv, self.Hq // self.Hkv,
                                             max_splits=self.graph_plans[B][1])
            self.g_split.copy_(torch.tensor([split], dtype=torch.int32).pin_memory(), non_blocking=True)
        g.replay()
        if len(rows) == B and rows == list(range(B)):
            return lg
        return lg[torch.tensor(rows, dtype=torch.long).to(self.device, non_blocking=True)]
