"""Hybrid KV-cache manager: separate block pools for full-attention and
sliding-window layers (gpt-oss: 18 of 36 layers attend to the last 128 tokens
only). The reference runs its gpt-oss P/D decoders with vLLM's hybrid manager
(``--no-disable-hybrid-kv-cache-manager``,
guides/pd-disaggregation/modelserver/gpu/vllm/base/patch-decode.yaml:19).

Without it every layer keeps the whole context, so a windowed layer holds
~40x more KV than it can ever read at ISL 5000. Here:

* the full-attention layers live in the main pool (``runner.kv``, the block
  manager ``full``: prefix caching, KV events, metrics as before);
* the windowed layers live in their own, much smaller pool
  (``runner.kv_swa``, block manager ``swa`` with a reserved null block 0):
  after every step each running sequence releases the windowed blocks that lie
  entirely before the first key any of its future queries can attend
  (``release_before(num_computed - window + 1)``); released entries point at
  the null block, which the window-limited attention kernels never read;
* released blocks stay content-addressed in the windowed pool's LRU, so a
  prefix-cache hit needs only the LAST window of the prefix there
  (``acquire_window``); the hit is the longest prefix both groups hold;
* P/D (kvx): the prefiller holds both groups' tables (``transfer_tables``; the
  windowed one is null before the last window), the decoder allocates the full
  prompt in the full group and the last window in the windowed group
  (``allocate_remote``), and the pull copies each group's non-null blocks.

The windowed pool is sized for every sequence's window plus one step's prefill
chunks (``swa_blocks``); the full pool gets the rest of the KV budget, so
capacity in tokens grows by ~ L / L_full (1.9x for gpt-oss at
--gpu-memory-utilization fixed).

The scheduler sees the BlockManager interface: ``grow`` is all-or-nothing over
both groups (it fails, changing neither, if either cannot grow, so preemption
follows whichever pool is exhausted) and ``can_allocate`` checks both; block
counts reported to metrics / the router are the full group's.
"""
from __future__ import annotations

import math


def swa_blocks(max_num_seqs: int, max_num_batched_tokens: int, window: int, block_size: int) -> int:
    """Windowed-pool size: per running sequence the blocks a window can span plus
    the one being written, plus one step's prefill chunks (their blocks exist
    until the step ends), plus the null block and slack for partial blocks."""
    per_seq = math.ceil((window - 1) / block_size) + 2
    return max_num_seqs * per_seq + math.ceil(max_num_batched_tokens / block_size) + max_num_seqs + 1


class HybridBlockManager:
    def __init__(self, rt, num_full_blocks: int, num_swa_blocks: int, block_size: int, window: int,
                 prefix_caching: bool, emit_events: bool, swa_events: bool = False):
        self.full = rt.BlockManager(num_full_blocks, block_size, prefix_caching, emit_events)
        # windowed-group events feed the offload tier only (never published to the router)
        self.swa = rt.BlockManager(num_swa_blocks, block_size, prefix_caching, swa_events, 1)
        self.window = window
        self.block_size = block_size
        self.num_blocks = self.full.num_blocks

    # ---- admission / prefix cache
    def lookup(self, toks, extra) -> int:
        return self.full.lookup(toks, extra)

    def acquire(self, seq_id, toks, extra) -> int:
        hit = self.full.lookup(toks, extra)
        hit = self.swa.acquire_window(seq_id, toks, extra, hit, self.window)
        got = self.full.acquire(seq_id, toks, extra, hit)
        assert got == hit, (got, hit)
        return hit

    def can_allocate(self, n: int) -> bool:
        # a new sequence's first blocks come from BOTH pools (the windowed table
        # grows with the sequence and nulls its head only after each step)
        return self.full.can_allocate(n) and self.swa.can_allocate(n)

    def grow(self, seq_id, total_tokens: int) -> bool:
        """All or nothing over both pools: when either cannot grow, neither does,
        so the scheduler preempts on whichever pool is exhausted (a failed
        windowed grow must not leave the full pool's new blocks behind)."""
        nb = -(-total_tokens // self.block_size)
        need_full = nb - self.full.num_seq_blocks(seq_id)
        need_swa = nb - self.swa.num_seq_blocks(seq_id)
        if need_full > self.full.num_free() or need_swa > self.swa.num_free():
            return False
        ok = self.full.grow(seq_id, total_tokens) and self.swa.grow(seq_id, total_tokens)
        assert ok, "hybrid grow: pool changed between the check and the grow"
        return True

    def commit(self, seq_id, toks, num_computed: int):
        self.full.commit(seq_id, toks, num_computed)
        self.swa.commit(seq_id, toks, num_computed)

    def after_compute(self, seq_id, num_computed: int) -> int:
        """Release windowed blocks no future query of this sequence can attend."""
        return self.swa.release_before(seq_id, num_computed - self.window + 1)

    def free(self, seq_id):
        self.full.free(seq_id)
        self.swa.free(seq_id)

    def allocate_remote(self, seq_id, num_tokens, extra):
        """P/D decode side: fresh blocks for the whole prompt in the full group, and
        in the windowed group only for the last window (earlier entries null) -
        the prefiller holds exactly those (it released the rest after its step)."""
        full = self.full.allocate_remote(seq_id, num_tokens, extra)
        if not full:
            return []
        swa = self.swa.allocate_remote(seq_id, num_tokens, extra, self.window)
        if not swa and num_tokens > 0:
            self.full.free(seq_id)
            return []
        return HybridBlocks(full, swa)

    def transfer_tables(self, seq_id):
        """Both groups' tables of a finished prefill (P side of P/D)."""
        return HybridBlocks(self.full.block_table(seq_id), self.swa.block_table(seq_id))

    # ---- tables
    def has_seq(self, seq_id) -> bool:
        return self.full.has_seq(seq_id)

    def block_table(self, seq_id):
        return self.full.block_table(seq_id)

    def block_table_swa(self, seq_id):
        return self.swa.block_table(seq_id)

    def num_seq_blocks(self, seq_id) -> int:
        return self.full.num_seq_blocks(seq_id)

    def fill_block_tables(self, ids, out):
        self.full.fill_block_tables(ids, out)

    # ---- accounting / events (full group: what the router and metrics see)
    def num_free(self) -> int:
        return self.full.num_free()

    def num_cached(self) -> int:
        return self.full.num_cached()

    def usage(self) -> float:
        return max(self.full.usage(), self.swa.usage())

    def reset_prefix_cache(self):
        self.full.reset_prefix_cache()
        self.swa.reset_prefix_cache()

    def take_events(self):
        return self.full.take_events()

    def take_swa_events(self):
        return self.swa.take_events()

    def take_evicted(self):
        return self.full.take_evicted()

    def prefix_stats(self):
        return self.full.prefix_stats()

    def cached_block_for(self, h):
        return self.full.cached_block_for(h)

    def check_invariants(self):
        self.full.check_invariants()
        self.swa.check_invariants()


class HybridTables(dict):
    """seq_id -> full-group block table, with the windowed group's tables in ``swa``."""

    def __init__(self, full: dict, swa: dict):
        super().__init__(full)
        self.swa = swa


class HybridBlocks(list):
    """A full-group block list carrying the windowed group's list in ``swa``
    (null entries = block 0): what kvx moves for one request of a hybrid cache."""

    def __init__(self, full, swa):
        super().__init__(full)
        self.swa = list(swa)
