"""Continuous-batching scheduler with chunked prefill, APC and preemption.

One token budget per step (``max_num_batched_tokens``) shared by decodes and
prefill chunks (vLLM-v1 style "unified" scheduling, the behaviour the
reference's recipes tune with ``--max-num-batched-tokens`` / ``--max-num-seqs``,
SURVEY C22 and §5.7 item 1):

1. running requests, in arrival/priority order: decodes take 1 token, partial
   prefills continue with the next chunk;
2. waiting requests are admitted (prefix-cache lookup first) while budget,
   KV blocks and ``max_num_seqs`` allow;
3. when the KV pool is exhausted the lowest-priority, most recent running
   request is preempted (recompute mode: its blocks are freed).

P/D hooks: requests with ``kv_transfer_params.do_remote_prefill`` wait in
WAITING_FOR_REMOTE_KV until the connector reports their KV landed; requests
with ``do_remote_decode`` keep their blocks after finishing until the decode
side releases them (or a timeout), see ``llmd_amd.kvx.connector``.
"""
from __future__ import annotations

import heapq
import itertools
import os
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from .config import EngineConfig
from .request import Request, Status

# GEMM alignment may not trim a chunk that finishes its prompt (engine/scheduler._align_tokens)
KEEP_FINAL_CHUNK = os.environ.get("LLMD_ALIGN_KEEP_FINAL", "1") == "1"


@dataclass
class ScheduledReq:
    req: Request
    num_new_tokens: int
    start: int  # num_computed_tokens before this step

    @property
    def is_decode(self) -> bool:
        return self.num_new_tokens == 1

    @property
    def samples(self) -> bool:
        return self.start + self.num_new_tokens >= self.req.num_tokens


@dataclass
class SchedulerOutput:
    decodes: list[ScheduledReq] = field(default_factory=list)
    prefills: list[ScheduledReq] = field(default_factory=list)
    preempted: list[Request] = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        return len(self.decodes) + sum(s.num_new_tokens for s in self.prefills)

    @property
    def empty(self) -> bool:
        return not self.decodes and not self.prefills

    def all(self) -> list[ScheduledReq]:
        return self.decodes + self.prefills


class _WaitQueue:
    """FCFS deque or (priority, arrival) heap; lower priority value first is
    NOT the vLLM convention - here higher `priority` = more important."""

    def __init__(self, policy: str):
        self.policy = policy
        self.dq: deque[Request] = deque()
        self.heap: list = []
        self._c = itertools.count()

    def push(self, r: Request, front: bool = False):
        if self.policy == "priority":
            heapq.heappush(self.heap, (-r.priority, r.arrival_time, next(self._c), r))
        elif front:
            self.dq.appendleft(r)
        else:
            self.dq.append(r)

    def peek(self) -> Optional[Request]:
        if self.policy == "priority":
            return self.heap[0][3] if self.heap else None
        return self.dq[0] if self.dq else None

    def pop(self) -> Request:
        if self.policy == "priority":
            return heapq.heappop(self.heap)[3]
        return self.dq.popleft()

    def remove(self, r: Request) -> bool:
        if self.policy == "priority":
            for i, e in enumerate(self.heap):
                if e[3] is r:
                    self.heap.pop(i)
                    heapq.heapify(self.heap)
                    return True
            return False
        try:
            self.dq.remove(r)
            return True
        except ValueError:
            return False

    def __len__(self):
        return len(self.heap) if self.policy == "priority" else len(self.dq)

    def __iter__(self):
        # iterate over a snapshot: callers may remove entries while iterating
        if self.policy == "priority":
            return iter([e[3] for e in sorted(self.heap)])
        return iter(list(self.dq))


class Scheduler:
    def __init__(self, cfg: EngineConfig, block_manager, connector=None):
        self.cfg = cfg
        self.sc = cfg.sched
        self.bm = block_manager
        self.bs = block_manager.block_size
        self.connector = connector
        self.offload = None  # set by the engine when a KV offload tier is configured
        self.waiting = _WaitQueue(self.sc.policy)
        self.running: list[Request] = []
        self.remote_wait: dict[str, Request] = {}
        # reloading their prefix from the offload tiers (kvcache/offload.py start_load / poll_loads)
        self.offload_wait: dict[str, Request] = {}
        # aborted while their KV pull was in flight: request id -> seq id whose
        # blocks stay allocated until the connector reports the pull finished
        self.aborted_remote: dict[str, int] = {}
        self.requests: dict[str, Request] = {}
        self.eos = set(cfg.model_config.eos_ids)
        self.num_preemptions_total = 0
        self.errored: list[Request] = []  # finished by the scheduler itself (not via update)
        self._window_release = hasattr(block_manager, "after_compute")
        self._tok_arrays: dict[str, np.ndarray] = {}

    # ------------------------------------------------------------ admission
    def add_request(self, req: Request):
        if req.request_id in self.requests:
            raise ValueError(f"duplicate request id {req.request_id}")
        if req.num_prompt_tokens == 0:
            raise ValueError("empty prompt")
        if req.num_prompt_tokens + 1 > self.sc.max_model_len:
            raise ValueError(f"prompt ({req.num_prompt_tokens} tokens) exceeds max_model_len {self.sc.max_model_len}")
        self.requests[req.request_id] = req
        ktp = req.kv_transfer_params or {}
        if ktp.get("do_remote_prefill") and self.connector is not None:
            req.status = Status.WAITING_FOR_REMOTE_KV
        self.waiting.push(req)

    def abort(self, request_id: str) -> Optional[Request]:
        r = self.requests.get(request_id)
        if r is None or r.status.finished:
            return None
        if r in self.running:
            self.running.remove(r)
        elif request_id in self.offload_wait:
            # the side stream may still be scattering into its blocks: they are freed
            # when the load reports done (schedule -> poll_loads)
            self.offload.cancel_load(request_id)
            self._finish(r, Status.FINISHED_ABORTED, free_blocks=False)
            return r
        elif self.remote_wait.pop(request_id, None) is not None:
            # the transfer worker may still be writing into this request's local
            # blocks: keep them allocated until the pull reports done
            self.connector.cancel_load(request_id)
            self.aborted_remote[request_id] = r.seq_id
            self._finish(r, Status.FINISHED_ABORTED, free_blocks=False)
            return r
        else:
            self.waiting.remove(r)
        self._finish(r, Status.FINISHED_ABORTED)
        return r

    @property
    def num_waiting(self) -> int:
        return len(self.waiting) + len(self.remote_wait) + len(self.offload_wait)

    @property
    def num_running(self) -> int:
        return len(self.running)

    def has_work(self) -> bool:
        return (bool(self.running) or len(self.waiting) > 0 or bool(self.remote_wait)
                or bool(self.aborted_remote) or bool(self.offload_wait))

    # ------------------------------------------------------------ helpers
    def _tokens(self, r: Request) -> np.ndarray:
        return np.asarray(r.all_token_ids, dtype=np.int32)

    def _preempt(self, victim: Request, out: SchedulerOutput):
        self.running.remove(victim)
        self.bm.free(victim.seq_id)
        victim.num_computed_tokens = 0
        victim.num_preemptions += 1
        victim.status = Status.PREEMPTED
        self.num_preemptions_total += 1
        self.waiting.push(victim, front=True)
        out.preempted.append(victim)

    def _unschedule(self, victim: Request, out: SchedulerOutput) -> int:
        for lst in (out.decodes, out.prefills):
            for k, sr in enumerate(lst):
                if sr.req is victim:
                    lst.pop(k)
                    return sr.num_new_tokens
        return 0

    def _pick_victim(self) -> Request:
        if self.sc.policy == "priority":
            return min(self.running, key=lambda r: (r.priority, -r.arrival_time))
        return self.running[-1]

    # ------------------------------------------------------------ schedule
    def schedule(self) -> SchedulerOutput:
        out = SchedulerOutput()
        budget = self.sc.max_num_batched_tokens
        # 0. remote-KV arrivals (P/D decode side)
        if self.connector is not None:
            for rid in self.connector.poll_finished_recv():
                seq = self.aborted_remote.pop(rid, None)
                if seq is not None:
                    self.connector.recv_ok(rid)  # drop the result
                    self.bm.free(seq)
                    continue
                r = self.remote_wait.pop(rid, None)
                if r is None:
                    continue
                ok = self.connector.recv_ok(rid)
                if ok:
                    # all prompt tokens but the last are in the cache; the last one is
                    # recomputed locally to produce the first output token's logits
                    r.num_computed_tokens = r.num_prompt_tokens - 1
                    r.num_cached_tokens = r.num_computed_tokens
                    r.status = Status.RUNNING
                    self.running.append(r)
                else:
                    policy = (self.cfg.kv_transfer_config or {}).get("kv_load_failure_policy", "recompute")
                    if policy == "fail":
                        self.bm.free(r.seq_id)
                        self._finish(r, Status.FINISHED_ERROR)
                        self.errored.append(r)
                        continue
                    self.bm.free(r.seq_id)
                    r.num_computed_tokens = 0
                    r.status = Status.WAITING
                    r.kv_transfer_params = None
                    self.waiting.push(r, front=True)
        # 0b. offload-tier reloads that landed: back to the head of the queue with the
        # reloaded tokens counted as computed
        if self.offload_wait:
            for r, ntok in self.offload.poll_loads():
                if self.offload_wait.pop(r.request_id, None) is None:
                    continue
                if r.status.finished:  # aborted while loading
                    self.bm.free(r.seq_id)
                    continue
                r.num_computed_tokens += ntok
                if r.num_preemptions == 0:
                    r.num_cached_tokens = r.num_computed_tokens
                self.waiting.push(r, front=True)
        # 1. running
        i = 0
        while i < len(self.running) and budget > 0:
            r = self.running[i]
            n = r.num_tokens - r.num_computed_tokens
            if n <= 0 or r.final_pending:  # final_pending: its last token is in flight (async)
                i += 1
                continue
            n = min(n, budget)
            if self.sc.long_prefill_token_threshold and n > 1:
                n = min(n, self.sc.long_prefill_token_threshold)
            self_preempted = False
            while not self.bm.grow(r.seq_id, r.num_computed_tokens + n):
                victim = self._pick_victim()
                vidx = self.running.index(victim)
                budget += self._unschedule(victim, out)
                self._preempt(victim, out)
                if victim is r:
                    self_preempted = True
                    break
                if vidx < i:
                    i -= 1
            if self_preempted:
                continue  # r left `running`; index i now points at the next request
            sr = ScheduledReq(r, n, r.num_computed_tokens)
            (out.decodes if sr.is_decode else out.prefills).append(sr)
            budget -= n
            i += 1
        # 2. waiting
        while (budget > 0 and not out.preempted and len(self.waiting) > 0
               and len(self.running) < self.sc.max_num_seqs):
            r = self.waiting.peek()
            if r.status == Status.WAITING_FOR_REMOTE_KV:
                # allocate destination blocks and start the pull
                blocks = self.bm.allocate_remote(r.seq_id, r.num_prompt_tokens, r.cache_extra)
                if not blocks:
                    break
                self.waiting.pop()
                self.remote_wait[r.request_id] = r
                if r.first_scheduled_time is None:
                    r.first_scheduled_time = time.monotonic()
                self.connector.start_load(r, blocks)
                continue
            if not self.bm.has_seq(r.seq_id):
                toks = self._tokens(r)
                cached = self.bm.acquire(r.seq_id, toks, r.cache_extra)
                r.num_computed_tokens = cached
                if r.num_preemptions == 0:
                    r.num_cached_tokens = cached
                if (self.offload is not None and self.cfg.cache.enable_prefix_caching and self.running
                        and self._reload_cannot_fit(r, cached, budget)):
                    # it would have to give the reloaded blocks back at once (below) and
                    # reload them again next step: wait holding nothing until blocks free up
                    self.bm.free(r.seq_id)
                    r.num_computed_tokens = 0
                    break
                if (self.offload is not None and self.cfg.cache.enable_prefix_caching
                        and self.offload.start_load(r, toks, cached, self.bm)):
                    # host / disk blocks continue the prefix: they load asynchronously
                    # (side stream, native read pool) while the engine keeps stepping
                    self.waiting.pop()
                    self.offload_wait[r.request_id] = r
                    if r.first_scheduled_time is None:
                        r.first_scheduled_time = time.monotonic()
                    continue
            n = r.num_tokens - r.num_computed_tokens
            if not self.sc.enable_chunked_prefill and n > budget:
                break
            n = min(n, budget)
            if self.sc.long_prefill_token_threshold and n > 1:
                n = min(n, self.sc.long_prefill_token_threshold)
            if not self.bm.grow(r.seq_id, r.num_computed_tokens + n):
                if not self.running:
                    # nothing to preempt and still no room: cannot make progress
                    if self.bm.num_free() == self.bm.num_blocks - self.bm.num_seq_blocks(r.seq_id):
                        self.waiting.pop()
                        self.bm.free(r.seq_id)
                        self._finish(r, Status.FINISHED_ERROR)
                        self.errored.append(r)
                        continue
                else:
                    # wait holding nothing: a waiting request that keeps its prefix (or
                    # host-reloaded) blocks can starve a preempted request queued ahead
                    # of it, and neither ever runs. Its next admission re-acquires the
                    # prefix (GPU cache, then host tier).
                    self.bm.free(r.seq_id)
                    r.num_computed_tokens = 0
                break
            self.waiting.pop()
            r.status = Status.RUNNING
            if r.first_scheduled_time is None:
                r.first_scheduled_time = time.monotonic()
            self.running.append(r)
            sr = ScheduledReq(r, n, r.num_computed_tokens)
            (out.decodes if sr.is_decode else out.prefills).append(sr)
            budget -= n
        self._align_tokens(out)
        return out

    def _reload_cannot_fit(self, r, cached: int, budget: int) -> bool:
        """True when the pool cannot hold this request's first chunk even after a
        tier reload (the blocks it holds now plus the free ones): reloading host /
        disk blocks it must release in the same step only repeats every step."""
        bs = self.bm.block_size
        want = -(-min(r.num_tokens, cached + max(budget, 1)) // bs)
        return want - self.bm.num_seq_blocks(r.seq_id) > self.bm.num_free()

    def _align_tokens(self, out: SchedulerOutput) -> None:
        """Trim prefill chunks, newest first, so the step's token count is a
        multiple of ``prefill_token_align`` (GEMM-friendly M). With
        ``LLMD_ALIGN_KEEP_FINAL=1`` only chunks that do not finish their prompt
        give tokens up (trimming a FINAL chunk adds a whole extra step for its
        tail: a 5000-token prompt beside 64 decodes becomes 4608- and 518-token
        steps, 509 + 103 ms). On by default since round 5: the unaligned 5064-row GEMMs
        that hipBLASLt runs ~20 % slower per token (profiles/gemm_prefill_odd_m.txt) go
        to the hand-written prefill GEMM through ops/pgemm_table.py (o / down 28-38 %,
        qkv 11 %, fused gate/up + SiLU 6 % faster than hipBLASLt there,
        profiles/pgemm_r5_v3_v6_5064.txt), so one 5064-token step replaces the 4608 + 518
        pair. LLMD_ALIGN_KEEP_FINAL=0 restores trimming final chunks too. Each
        trimmed chunk keeps at least two tokens (a one-token chunk would read as
        a decode); steps below two alignment units, or whose chunks cannot give
        up the whole remainder, run as scheduled. Trimmed tokens go in the next
        step (their blocks stay allocated, so the next ``grow`` is a no-op)."""
        a = self.sc.prefill_token_align
        if a <= 0 or not out.prefills:
            return
        total = out.num_tokens
        rem = total % a
        if total < 2 * a or rem == 0:
            return

        def slack(sr):
            if KEEP_FINAL_CHUNK and sr.start + sr.num_new_tokens >= sr.req.num_tokens:  # final: keep whole
                return 0
            return max(sr.num_new_tokens - 2, 0)

        if sum(slack(sr) for sr in out.prefills) < rem:
            return
        for sr in reversed(out.prefills):
            take = min(rem, slack(sr))
            sr.num_new_tokens -= take
            rem -= take
            if rem == 0:
                break

    def update(self, out: SchedulerOutput, sampled: dict[int, tuple[int, float]]) -> list[Request]:
        """Apply a step's results. `sampled`: seq_id -> (token, logprob).
        Returns requests that produced new tokens or finished this step."""
        touched = []
        now = time.monotonic()
        bs = self.cfg.cache.block_size
        for sr in out.all():
            r = sr.req
            if r.status.finished:
                continue
            r.num_computed_tokens = sr.start + sr.num_new_tokens
            # hash/register newly completed blocks only (a decode completes one
            # every block_size steps; converting the whole context each step cost
            # O(ctx) host time per request)
            if (self.cfg.cache.enable_prefix_caching and r.num_computed_tokens // bs > sr.start // bs
                    and self.bm.has_seq(r.seq_id)):
                self.bm.commit(r.seq_id, self._tokens(r), r.num_computed_tokens)
            if self._window_release and self.bm.has_seq(r.seq_id):
                # hybrid KV cache: windowed blocks no future query can reach go back to the pool.
                # A P/D prefill keeps one key more: the decoder recomputes the last prompt
                # token, whose query reaches back to position n - window (allocate_remote).
                n_keep = r.num_computed_tokens
                if (r.kv_transfer_params or {}).get("do_remote_decode"):
                    n_keep -= 1
                self.bm.after_compute(r.seq_id, n_keep)
            if r.seq_id in sampled:
                tok, lp = sampled[r.seq_id]
                r.output_token_ids.append(tok)
                r.output_logprobs.append(lp)
                if r.first_token_time is None:
                    r.first_token_time = now
                r.last_token_time = now
                self._check_stop(r)
                touched.append(r)
        return touched

    # ------------------------------------------------------------ async scheduling
    # A step's update split in two (engine.py async path): ``advance`` when the step is
    # launched - positions move on, completed blocks are committed, windowed blocks released,
    # and every sampling request gets a placeholder output token, so the next step can be
    # scheduled before this one's tokens reach the host; ``resolve`` once they have -
    # placeholders become the real tokens and stop conditions are checked.
    PLACEHOLDER = -1

    def advance(self, out: SchedulerOutput, sampling: set) -> None:
        """Called once the previous step is resolved, so every INPUT token of this step is
        real: blocks this step completes are committed here (hashes over their tokens),
        before the windowed pool releases anything (write-through offload sees them)."""
        bs = self.cfg.cache.block_size
        for sr in out.all():
            r = sr.req
            if r.status.finished:
                continue
            r.num_computed_tokens = sr.start + sr.num_new_tokens
            if (self.cfg.cache.enable_prefix_caching and r.num_computed_tokens // bs > sr.start // bs
                    and self.bm.has_seq(r.seq_id)):
                self.bm.commit(r.seq_id, self._tokens(r)[:r.num_computed_tokens], r.num_computed_tokens)
            if self._window_release and self.bm.has_seq(r.seq_id):
                # windowed blocks no later query reaches: released now (token values not needed;
                # a step launched after this one reuses them only after this one ran - one stream)
                n_keep = r.num_computed_tokens
                if (r.kv_transfer_params or {}).get("do_remote_decode"):
                    n_keep -= 1
                self.bm.after_compute(r.seq_id, n_keep)
            if r.seq_id in sampling:
                r.output_token_ids.append(self.PLACEHOLDER)
                r.output_logprobs.append(0.0)
                r.async_pending = True
                # the token in flight is the last one whatever its value: do not schedule again
                if len(r.output_token_ids) >= r.params.max_tokens or r.num_tokens >= self.sc.max_model_len:
                    r.final_pending = True

    def resolve(self, out: SchedulerOutput, sampled: dict[int, tuple[int, float]]) -> list[Request]:
        touched = []
        now = time.monotonic()
        for sr in out.all():
            r = sr.req
            if r.status.finished:
                continue
            if r.seq_id in sampled and r.async_pending:
                tok, lp = sampled[r.seq_id]
                r.output_token_ids[-1] = tok
                r.output_logprobs[-1] = lp
                r.async_pending = False
                if r.first_token_time is None:
                    r.first_token_time = now
                r.last_token_time = now
                self._check_stop(r)
                touched.append(r)
        return touched

    def _check_stop(self, r: Request):
        p = r.params
        n_out = len(r.output_token_ids)
        tok = r.output_token_ids[-1]
        if n_out >= p.min_tokens:
            if (not p.ignore_eos and tok in self.eos) or tok in p.stop_token_ids:
                r.stop_reason = tok
                return self._finish_running(r, Status.FINISHED_STOPPED)
        if n_out >= p.max_tokens or r.num_tokens >= self.sc.max_model_len:
            return self._finish_running(r, Status.FINISHED_LENGTH)

    def finish_stopped_by_string(self, r: Request):
        if not r.status.finished:
            self._finish_running(r, Status.FINISHED_STOPPED)

    def _finish_running(self, r: Request, status: Status):
        if r in self.running:
            self.running.remove(r)
        elif r.status == Status.PREEMPTED:  # async: preempted while its last token was in flight
            self.waiting.remove(r)
        self._finish(r, status)

    def _finish(self, r: Request, status: Status, free_blocks: bool = True):
        r.status = status
        r.finished_time = time.monotonic()
        ktp = r.kv_transfer_params or {}
        if ktp.get("do_remote_decode") and self.connector is not None and status != Status.FINISHED_ABORTED:
            # P side: keep blocks for the remote reader; the connector frees them
            tables = []
            if self.bm.has_seq(r.seq_id):
                tables = (self.bm.transfer_tables(r.seq_id) if hasattr(self.bm, "transfer_tables")
                          else self.bm.block_table(r.seq_id))
            self.connector.hold_for_remote(r, tables)
        elif free_blocks:
            self.bm.free(r.seq_id)
        self.requests.pop(r.request_id, None)

    def release_held(self, seq_id: int):
        self.bm.free(seq_id)
