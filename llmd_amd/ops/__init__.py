"""Op layer: HIP/CDNA4 kernels for GPU tensors, fp32 torch references for CPU.

GPU tensors ALWAYS go to the native ``llmd_amd._C`` library; if it is missing
on a GPU host the call raises (no silent eager fallback). CPU tensors use
``llmd_amd.ops.reference`` so the whole engine runs in CPU CI.
"""
from __future__ import annotations

import logging
import math
import os
from typing import Optional

import torch

from . import reference as ref

log = logging.getLogger("llmd.ops")

_C = None
_C_ERR: Exception | None = None


def native():
    """Return the loaded ``_C`` module, building/loading it on first use."""
    global _C, _C_ERR
    if _C is not None:
        return _C
    import importlib

    debug = os.environ.get("LLMD_KERNEL_DEBUG", "0") == "1"  # kernels with LLMD_DCHECK assertions
    name = "llmd_amd._C_debug" if debug else "llmd_amd._C"
    try:
        mod = importlib.import_module(name)
    except ImportError as e:  # pragma: no cover - exercised on GPU hosts only
        _C_ERR = e
        if os.environ.get("LLMD_AUTOBUILD", "1") == "1":
            from llmd_amd.build import build_ops

            build_ops(debug=debug)
            mod = importlib.import_module(name)
        else:
            raise RuntimeError(f"{name} HIP extension not built: {e}") from e
    _C = mod
    return _C


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ---------------------------------------------------------------- norms
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    if not _gpu(x):
        r = ref.rms_norm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty_like(x)
    native().rms_norm(out, x, w, eps)
    return out


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """residual += x; x = rmsnorm(residual) * w (both in place)."""
    if not _gpu(x):
        ref.fused_add_rms_norm(x, residual, w, eps)
        return
    native().fused_add_rms_norm(x, residual, w, eps)


def qk_rms_norm(qkv: torch.Tensor, qw: torch.Tensor, kw: torch.Tensor, Hq: int, Hkv: int, eps: float):
    """Qwen3 per-head RMSNorm of the q and k heads, in place in the fused QKV
    projection output ``qkv[T, (Hq + 2 Hkv) * D]`` (one kernel, no strided copies)."""
    if not _gpu(qkv):
        D = qw.numel()
        T = qkv.shape[0]
        q = qkv[:, : Hq * D].reshape(T * Hq, D)
        k = qkv[:, Hq * D: (Hq + Hkv) * D].reshape(T * Hkv, D)
        qkv[:, : Hq * D] = ref.rms_norm(q, qw, eps).view(T, -1)
        qkv[:, Hq * D: (Hq + Hkv) * D] = ref.rms_norm(k, kw, eps).view(T, -1)
        return qkv
    native().qk_rms_norm(qkv, qw, kw, Hq, Hkv, eps)
    return qkv


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float):
    if not _gpu(x):
        return ref.layer_norm(x, w, b, eps)
    out = torch.empty_like(x)
    native().layer_norm(out, x, None, w, b, eps)
    return out


def fused_add_layer_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float):
    """residual += x; x = layernorm(residual) * w + b (both in place)."""
    if not _gpu(x):
        ref.fused_add_layer_norm(x, residual, w, b, eps)
        return
    native().layer_norm(x, x, residual, w, b, eps)


# ---------------------------------------------------------------- rope + cache
def rope_cache(qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache, neox=True, k_scale=1.0,
               v_scale=1.0):
    """RoPE + paged KV write; bf16 or fp8 e4m3fn caches (fp8 stores x / scale)."""
    if not _gpu(qkv):
        ref.rope_cache(qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache, neox, k_scale, v_scale)
        return
    native().rope_cache(qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache, neox, k_scale, v_scale)


# ---------------------------------------------------------------- activation
ACT_SILU, ACT_GELU_TANH, ACT_SWIGLU_OAI = 0, 1, 2


def gated_act(x: torch.Tensor, mode: int = ACT_SILU, alpha: float = 1.702, limit: float = 7.0,
              out: torch.Tensor | None = None):
    if not _gpu(x):
        r = ref.gated_act(x, mode, alpha, limit)
        if out is not None:
            out.copy_(r)
            return out
        return r
    F = x.shape[1] // 2
    if out is None:
        out = torch.empty(x.shape[0], F, dtype=x.dtype, device=x.device)
    native().gated_act(out, x, mode, alpha, limit)
    return out


# ---------------------------------------------------------------- attention
def prefill_tokens_per_item(Hq: int, Hkv: int, D: int = 128, block_size: int = 64, fp8: bool = False) -> int:
    """Query tokens per prefill work item of the kernel the native dispatcher
    picks for these arguments (the native helper is the single source)."""
    try:
        return int(native().prefill_tokens_per_item(Hq, Hkv, D, block_size, fp8))
    except (ImportError, OSError):  # CPU-only environment: the reference path ignores items
        G = Hq // Hkv
        hpw = 4 if G % 4 == 0 else (2 if G % 2 == 0 else 1)
        return 32 * (4 // hpw)


def decode_split_plan(max_ctx: int, batch: int, Hkv: int, G: int, num_cus: int = 256,
                      min_split: int = 256, max_splits: Optional[int] = None) -> tuple[int, int]:
    """Pick (split_size, nsplit) for the decode kernel by a makespan model:
    batch x head-groups x nsplit workgroups run in rounds of two per CU, a
    round lasts as long as one split (its keys), plus a small per-split cost
    (partials + reduce). Splits are multiples of 64 keys and at least
    `min_split` when there is more than one. Measured (profiles/decode_nsplit.txt):
    batch 48 at 7.4k context 293 -> 264 us with 4 splits instead of 2 (1536
    workgroups = 3 full rounds rather than 768 = 1.5)."""
    ng = (G + 15) // 16
    base = max(1, batch * Hkv * ng)
    slots = 2 * num_cus
    ctx = max(1, max_ctx)
    hi = max(1, math.ceil(ctx / min_split))
    if max_splits is not None:
        hi = max(1, min(hi, max_splits))
    best = None
    for n in range(1, min(hi, 64) + 1):
        split = max(64, math.ceil(ctx / n / 64) * 64)
        n_eff = math.ceil(ctx / split)
        w = base * n_eff
        # up to two rounds the last one's idle slots are lost; beyond, workgroups of
        # uneven sequences finish at different times and the tail shrinks
        rounds = math.ceil(w / slots) if w <= 2 * slots else w / slots
        cost = rounds * split + 16 * n_eff
        if best is None or cost < best[0]:
            best = (cost, split, n_eff)
    return best[1], best[2]


class SharedPrefixPlan:
    """Shared-prefix ("cascade") decode plan for one step (SURVEY K01 on the
    prefix-cache workloads: many running sequences whose first blocks are the
    same physical KV blocks).

    sstart[b]   end of sequence b's shared prefix (0 = none): its own decode
                pass covers keys [sstart[b], L)
    pcount[b]   prefix partial slots written for b (one per work unit of its item)
    members     sequence indices, item by item (contiguous)
    work        int32 [nwork, 5] = (first member, members, key lo, key hi, slot
                offset); rows with 0 members are padding
    items       number of prefix items (groups of <= CASCADE_MEMBERS[np](G) members)
    np          prefix kernel variant (cascade_variant): 1 / 2 register kernel with
                1 / 2 16-column passes, 3 LDS-DMA kernel
    """

    __slots__ = ("sstart", "pcount", "members", "work", "items", "np", "max_slots")

    def __init__(self, sstart, pcount, members, work, items, np_, max_slots):
        self.sstart, self.pcount, self.members, self.work = sstart, pcount, members, work
        self.items, self.np, self.max_slots = items, np_, max_slots

    @property
    def work_units(self) -> int:
        return int((self.work[:, 1] > 0).sum())


def cascade_variant(G: int, D: int, bs: int, fp8: bool) -> Optional[int]:
    """Shared-prefix kernel for this geometry: 3 = LDS-DMA kernel (bf16 cache,
    G 4 or 8, D 64/128, block size >= 8; up to 128/G members per item),
    1 = register kernel (16/G members), 2 = its two-pass form (G = 16: 2
    members), None = no cascade (16 % G != 0)."""
    if not fp8 and G in (4, 8) and D in (64, 128) and bs >= 8:
        return 3
    if G < 16 and 16 % G == 0:
        return 1
    if G == 16:
        return 2  # one member per 16-column pass: two passes to pair sequences
    return None


CASCADE_MEMBERS = {1: lambda G: 16 // G, 2: lambda G: 32 // G, 3: lambda G: 128 // G}


def shared_prefix_plan(block_tables, seq_lens, bs: int, G: int, Hkv: int = 8, *, variant: int = 1,
                       max_slots: int = 16, min_prefix: int = 512, max_work: Optional[int] = None,
                       min_chunk: int = 512) -> Optional[SharedPrefixPlan]:
    """Group the decode batch by shared leading physical blocks.

    Only FULL blocks strictly before a sequence's current token count (the
    prefix cache shares full blocks; the current token's block is private).
    Members of a group are sorted by how many blocks they share with the
    group's first member and cut into items of at most the kernel variant's
    member capacity (CASCADE_MEMBERS); an item's prefix is the shortest shared
    run among its members. Items are split into work units of >= min_chunk
    keys, one round of workgroups over the chip in total (512 / Hkv units; 256 /
    Hkv for the one-workgroup-per-CU variant 2), at most `max_slots` per item.
    Returns None when nothing is shared (the plain kernel runs)."""
    import numpy as np

    if G > 16 or 16 % G:
        return None
    lens = np.asarray(seq_lens, dtype=np.int64)
    B = len(lens)
    if B < 2:
        return None
    bt = np.asarray(block_tables)[:B]
    cap = CASCADE_MEMBERS[variant](G)
    nfull = np.maximum((lens - 1) // bs, 0)
    min_blocks = max(1, -(-min_prefix // bs))
    elig = np.nonzero(nfull >= min_blocks)[0]
    if len(elig) < 2:
        return None
    # group by first physical block (sorted), LCP of every row with its group's
    # first row in one vectorised compare
    first = bt[elig, 0]
    order = np.argsort(first, kind="stable")
    elig, first = elig[order], first[order]
    _, gstart, gcount = np.unique(first, return_index=True, return_counts=True)
    multi = gcount >= 2
    if not multi.any():
        return None
    w = int(nfull[elig].max())
    leader = np.repeat(gstart, gcount)
    rows = bt[elig, :w]
    eq = rows == rows[leader]
    lcp = np.where(eq.all(1), w, eq.argmin(1))
    lcp = np.minimum(lcp, nfull[elig])
    items = []  # (prefix tokens, [members])
    for g0, n0 in zip(gstart[multi].tolist(), gcount[multi].tolist()):
        gl = lcp[g0:g0 + n0]
        o = np.argsort(-gl, kind="stable")
        o = o[gl[o] >= min_blocks]
        n = len(o)
        if n < 2:
            continue
        mem_sorted = elig[g0:g0 + n0][o].tolist()
        lcp_sorted = gl[o].tolist()
        nit = -(-n // cap)
        sizes = [n // nit + (1 if k < n % nit else 0) for k in range(nit)]
        pos = 0
        for sz in sizes:
            if sz >= 2:
                items.append((min(lcp_sorted[pos:pos + sz]) * bs, mem_sorted[pos:pos + sz]))
            pos += sz
    if not items:
        return None
    # one round of workgroups over the chip: variant 2 holds two passes'
    # accumulators (one workgroup per CU), the others run two per CU
    target = max(8, -(-(256 if variant == 2 else 512) // max(1, Hkv)))
    if max_work is not None:
        target = min(target, max_work)
    total = sum(p for p, _ in items)
    sstart = np.zeros(B, np.int32)
    pcount = np.zeros(B, np.int32)
    members = np.zeros(B, np.int32)
    work = []
    mpos = 0
    used_items = 0
    for P, mem in sorted(items, key=lambda x: -x[0] * len(x[1])):
        k = max(1, min(max_slots, round(target * P / total), -(-P // min_chunk)))
        split = -(-P // k)
        split = -(-split // 64) * 64
        k = -(-P // split)
        if max_work is not None and len(work) + k > max_work:
            continue  # no capacity left in the captured grid: these members run the plain path
        m0 = mpos
        for b in mem:
            members[mpos] = b
            mpos += 1
            sstart[b] = P
            pcount[b] = k
        for j in range(k):
            work.append((m0, len(mem), j * split, min(P, (j + 1) * split), j))
        used_items += 1
    if not work:
        return None
    nwork = len(work) if max_work is None else max_work
    wk = np.zeros((nwork, 5), np.int32)
    wk[:len(work)] = np.asarray(work, np.int32)
    return SharedPrefixPlan(sstart, pcount, members, wk, used_items, variant, max_slots)


def cascade_tensors(plan: SharedPrefixPlan, device, out: Optional[torch.Tensor] = None):
    """One int32 tensor [sstart | pcount | members | work] for paged_decode(cascade=...).
    ``out``: a static (hipGraph) buffer of the same layout to copy into."""
    import numpy as np

    flat = np.concatenate([plan.sstart, plan.pcount, plan.members, plan.work.reshape(-1)]).astype(np.int32)
    host = torch.from_numpy(flat)
    if out is not None:
        out[: host.numel()].copy_(host.pin_memory() if out.is_cuda else host, non_blocking=True)
        return (out[: host.numel()], plan.np, plan.max_slots)
    if torch.device(device).type == "cuda":
        host = host.pin_memory()
    return (host.to(device, non_blocking=True), plan.np, plan.max_slots)


def paged_decode(q, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale, window=0,
                 sinks=None, split=None, out=None, workspace=None, max_ctx=None, k_scale=1.0, v_scale=1.0,
                 cascade=None, split_dev=None):
    """q: [B, >=Hq*D] -> out [B, Hq*D]. k/v caches bf16 or fp8 e4m3fn (dequant scales).
    cascade: (tensor, np, max_slots) from cascade_tensors(shared_prefix_plan(...)): shared
    prefixes are read once per group by the prefix kernel; `split` must then cover the
    longest suffix (L - sstart), and the workspace holds nsplit + max_slots slots per row.
    split_dev: int32 [1] device tensor of keys per split read by the kernels instead of
    split[0] (a captured hipGraph re-sizes its splits per step; nsplit stays the grid)."""
    if not _gpu(q):
        r = ref.paged_decode(q, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale,
                             window, sinks, k_scale, v_scale)
        if out is not None:
            out.copy_(r)
            return out
        return r
    B = q.shape[0]
    if out is None:
        out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    if split is None:
        if max_ctx is None:
            max_ctx = int(seq_lens.max().item()) if B else 1
        if window and window > 0:
            max_ctx = min(max_ctx, window)
        split = decode_split_plan(max_ctx, B, Hkv, Hq // Hkv)
    split_size, nsplit = split
    ctens, cnp, nslot = None, 1, nsplit
    if cascade is not None and not (window and window > 0):
        ctens, cnp, extra = cascade
        nslot = nsplit + extra
    if nslot > 1:
        if workspace is None:
            part_o = torch.empty(B * Hq * nslot * D, dtype=torch.float32, device=q.device)
            part_ml = torch.empty(B * Hq * nslot * 2, dtype=torch.float32, device=q.device)
        else:
            part_o, part_ml = workspace
    else:
        part_o = part_ml = out.new_empty(0, dtype=torch.float32)
    native().paged_decode(out, q, k_cache, v_cache, block_tables, seq_lens, Hq, Hkv, D, scale,
                          window, sinks, split_size, nsplit, part_o, part_ml, k_scale, v_scale,
                          ctens, cnp, nslot, split_dev)
    return out


def build_prefill_items(q_len: list[int], ctx_len: list[int], tpi: int) -> list[tuple[int, int]]:
    """Work items (seq, first q token), heaviest (most keys) first."""
    items = []
    for s, (ql, cl) in enumerate(zip(q_len, ctx_len)):
        for t0 in range(0, ql, tpi):
            keys = cl - ql + min(ql, t0 + tpi)
            items.append((keys, s, t0))
    items.sort(key=lambda x: -x[0])
    return [(s, t0) for _, s, t0 in items]


# fp8-KV prefill through a bf16 copy of the step's blocks (kv_dequant_gather) and the bf16 v2 kernel
# instead of the fp8 v1 kernel (LLMD_PREFILL_FP8_VIA_BF16=0: the v1 fp8 kernel)
PREFILL_FP8_VIA_BF16 = os.environ.get("LLMD_PREFILL_FP8_VIA_BF16", "1") == "1"


def kv_dequant_gather(k_cache, v_cache, block_tables):
    """(k, v, table): the blocks ``block_tables`` [S, maxb] names in an fp8 paged cache [blocks, Hkv,
    bs, D], widened exactly to bf16 into dense copies [S * maxb, Hkv, bs, D] and the identity table
    over them (padding entries copy block 0, never read)."""
    S, mb = block_tables.shape
    shape = (S * mb,) + tuple(k_cache.shape[1:])
    if not _gpu(k_cache):
        ids = block_tables.reshape(-1).clamp(0, k_cache.shape[0] - 1).long()
        return (k_cache[ids].to(torch.bfloat16), v_cache[ids].to(torch.bfloat16),
                torch.arange(S * mb, dtype=torch.int32).view(S, mb))
    kd = torch.empty(shape, dtype=torch.bfloat16, device=k_cache.device)
    vd = torch.empty(shape, dtype=torch.bfloat16, device=k_cache.device)
    native().kv_dequant_gather(k_cache, v_cache, block_tables.contiguous(), kd, vd)
    return kd, vd, torch.arange(S * mb, dtype=torch.int32, device=k_cache.device).view(S, mb)


def paged_prefill(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, Hq, Hkv, D, scale,
                  window=0, sinks=None, items=None, out=None, k_scale=1.0, v_scale=1.0):
    if not _gpu(q):
        r = ref.paged_prefill(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, Hq, Hkv,
                              D, scale, window, sinks, k_scale, v_scale)
        if out is not None:
            out.copy_(r)
            return out
        return r
    if out is None:
        out = torch.empty(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    if (PREFILL_FP8_VIA_BF16 and k_cache.dtype == torch.float8_e4m3fn and k_cache.shape[-2] >= 16
            and D in (64, 128)):
        k_cache, v_cache, block_tables = kv_dequant_gather(k_cache, v_cache, block_tables)
    if items is None:
        tpi = prefill_tokens_per_item(Hq, Hkv, D, k_cache.shape[-2], k_cache.dtype == torch.float8_e4m3fn)
        it = build_prefill_items(q_len.tolist(), ctx_len.tolist(), tpi)
        items = torch.tensor(it, dtype=torch.int32).view(-1, 2).to(q.device, non_blocking=True)
    native().paged_prefill(out, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, items,
                           Hq, Hkv, D, scale, window, sinks, k_scale, v_scale)
    return out


# ---------------------------------------------------------------- fp8 linear (W8A8)
FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0


def quant_fp8_rows(x: torch.Tensor):
    """Dynamic per-token fp8: x [T, d] bf16 -> (q [T, d] e4m3fn, scale [T, 1] f32)."""
    if not _gpu(x):
        s = (x.float().abs().amax(1, keepdim=True) / FP8_MAX).clamp(min=1e-12)
        return (x.float() / s).clamp(-FP8_MAX, FP8_MAX).to(FP8), s
    x = x if x.stride(-1) == 1 and x.stride(0) % 8 == 0 else x.contiguous()
    q = torch.empty(x.shape, dtype=FP8, device=x.device)
    s = torch.empty(x.shape[0], 1, dtype=torch.float32, device=x.device)
    native().quant_fp8_rows(x, q, s)
    return q, s


def quant_fp8_weight(w: torch.Tensor):
    """Per-output-channel weight quantisation: w [N, K] -> (wq [N, K] e4m3fn, scale [1, N] f32)."""
    s = (w.float().abs().amax(1) / FP8_MAX).clamp(min=1e-12)
    wq = (w.float() / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return wq, s.view(1, -1).contiguous()


def rms_norm_quant(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None):
    """(q fp8 [T, d], scale [T, 1]) of rmsnorm(x [+ residual]) * w; with ``residual``
    it is updated in place (residual += x) like fused_add_rms_norm."""
    if not _gpu(x):
        if residual is not None:
            residual.copy_((residual.float() + x.float()).to(residual.dtype))
            y = ref.rms_norm(residual, w, eps)
        else:
            y = ref.rms_norm(x, w, eps)
        return quant_fp8_rows(y)
    q = torch.empty(x.shape, dtype=FP8, device=x.device)
    s = torch.empty(x.shape[0], 1, dtype=torch.float32, device=x.device)
    native().rms_norm_quant(q, s, x, residual, w, eps)
    return q, s


def gated_act_quant(x: torch.Tensor, mode: int = 0, alpha: float = 1.702, limit: float = 7.0):
    """(q fp8 [T, F], scale [T, 1]) of the gated activation (SURVEY K07 + K16)."""
    if not _gpu(x):
        return quant_fp8_rows(ref.gated_act(x, mode, alpha, limit))
    F = x.shape[1] // 2
    q = torch.empty(x.shape[0], F, dtype=FP8, device=x.device)
    s = torch.empty(x.shape[0], 1, dtype=torch.float32, device=x.device)
    native().gated_act_quant(q, s, x, mode, alpha, limit)
    return q, s


def fp8_linear(x, wq: torch.Tensor, w_scale: torch.Tensor, bias=None) -> torch.Tensor:
    """y = (q_x s_x) (q_w s_w)^T (+ bias), bf16 out. Activations are quantised
    per token on the fly (HIP kernel); the GEMM is hipBLASLt's fp8 GEMM with
    row-wise scales through torch._scaled_mm (a plain library GEMM).
    ``x`` may already be quantised: a (q, scale) pair from rms_norm_quant /
    gated_act_quant."""
    if isinstance(x, tuple):
        xq, xs = x
        if not _gpu(xq):
            y = (xq.float() * xs) @ (wq.float() * w_scale.view(-1, 1)).t()
            if bias is not None:
                y = y + bias.float()
            return y.to(torch.bfloat16)
        if xq.shape[0] == 0:
            return torch.empty(0, wq.shape[0], dtype=torch.bfloat16, device=xq.device)
        return _fp8_gemm(xq, xs, wq, w_scale, bias)
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    if not _gpu(x2):
        xq, xs = quant_fp8_rows(x2)
        y = (xq.float() * xs) @ (wq.float() * w_scale.view(-1, 1)).t()
        if bias is not None:
            y = y + bias.float()
        return y.to(torch.bfloat16).reshape(*lead, -1)
    if x2.shape[0] == 0:
        return x2.new_empty(0, wq.shape[0]).reshape(*lead, -1)
    xq, xs = quant_fp8_rows(x2)
    return _fp8_gemm(xq, xs, wq, w_scale, bias).reshape(*lead, -1)


def pgemm8_plan(M: int, N: int, K: int) -> Optional[bool]:
    """split_k of the fp8 prefill GEMM for this shape from the shipped table
    (ops/pgemm8_table.py), or None: hipBLASLt's scaled GEMM."""
    if PGEMM_AUTO == "0" or M < PGEMM_MIN_M:
        return None
    from .pgemm8_table import PGEMM8_TABLE

    e = PGEMM8_TABLE.get(((M + 255) // 256, N, K))
    return None if e is None else e[0]


def pgemm8_silu_planned(M: int, N: int, K: int) -> bool:
    """True where the shipped table has the SiLU-epilogue fp8 gate/up GEMM + a row
    quant ahead of GEMM + the fused act-quant kernel."""
    if PGEMM_AUTO == "0" or M < PGEMM_MIN_M:
        return False
    from .pgemm8_table import PGEMM8_TABLE

    e = PGEMM8_TABLE.get(("silu", (M + 255) // 256, N, K))
    return e is not None and e[0] is not None


def _fp8_gemm(xq, xs, wq, w_scale, bias):
    """Decode-sized M on the fp8 medium-M LDS-DMA GEMM where its measured table has it
    ahead of hipBLASLt's (tuned) scaled GEMM, prefill-sized M on the fp8 256 x 256
    tile GEMM (pgemm8) where its table does, else torch._scaled_mm."""
    if bias is None and _SKINNY and xq.is_contiguous() and wq.is_contiguous():
        plan = mgemm_fp8_choice(xq.shape[0], wq.shape[0], wq.shape[1])
        if plan is not None:
            return mgemm_fp8(xq, xs, wq, w_scale, plan)
        if pgemm_fp8_ok(xq, wq):
            sk = pgemm8_plan(xq.shape[0], wq.shape[0], wq.shape[1])
            if sk is not None:
                return pgemm_fp8(xq, xs, wq, w_scale, split_k=sk)
    return torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=w_scale, bias=bias, out_dtype=torch.bfloat16)


def pgemm_fp8(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor, epi: int = 0,
              out: Optional[torch.Tensor] = None, split_k: bool = True, persistent: bool = False) -> torch.Tensor:
    """Prefill fp8 W8A8 GEMM (csrc/ops/pgemm8.hip): (xs . xq) (ws . wq)^T in bf16,
    per-token xs [M(, 1)] and per-channel ws [(1, )N] fp32 scales; epi 3 =
    silu(gate) * up on wq = [gate; up] (output [M, N / 2]). N % 256 == 0,
    K % 128 == 0; ``split_k`` runs a last wave at most half full split over K
    (fp32 partials + a reduce); ``persistent`` (epi 0) walks the tiles as one K-step stream per
    workgroup (no per-tile prologue wait). Fails loudly without the native library."""
    M, N = xq.shape[0], wq.shape[0]
    if out is None:
        out = torch.empty(M, N // 2 if epi == 3 else N, dtype=torch.bfloat16, device=xq.device)
    native().pgemm_fp8(out, xq, xs, wq, ws, epi, split_k, persistent)
    return out


def pgemm_fp8_ok(xq: torch.Tensor, wq: torch.Tensor) -> bool:
    """Shapes / layouts the fp8 prefill GEMM takes."""
    return (xq.dim() == 2 and wq.dim() == 2 and wq.shape[0] % 256 == 0 and xq.shape[1] % 128 == 0
            and xq.stride(-1) == 1 and wq.stride(-1) == 1 and xq.stride(0) % 16 == 0 and wq.stride(0) % 16 == 0)


def pow2_ceil(r: torch.Tensor) -> torch.Tensor:
    """Smallest power of two >= r (f32, r > 0): the block scales of the fp8 MoE
    path are powers of two so the grouped GEMM passes them to the MFMA as E8M0
    exponents (csrc/include/llmd_common.h pow2_ceil)."""
    m, e = torch.frexp(r.float())
    return torch.ldexp(torch.ones_like(m), e - (m == 0.5).to(e.dtype))


def quant_fp8_groups(x: torch.Tensor, group: int = 128):
    """Per (token, 128-group) fp8: x [T, d] -> (q [T, d] e4m3fn, scale [T, ceil(d/128)] f32).
    Scales are powers of two (E8M0-exact)."""
    T, d = x.shape
    ng = (d + group - 1) // group
    if not _gpu(x):
        pad = ng * group - d
        xf = torch.nn.functional.pad(x.float(), (0, pad)).view(T, ng, group)
        s = pow2_ceil((xf.abs().amax(2) / FP8_MAX).clamp(min=1e-12))
        q = (xf / s[:, :, None]).clamp(-FP8_MAX, FP8_MAX).view(T, ng * group)[:, :d].to(FP8)
        return q, s
    assert group == 128
    x = x if x.stride(-1) == 1 and x.stride(0) % 8 == 0 else x.contiguous()
    q = torch.empty(x.shape, dtype=FP8, device=x.device)
    s = torch.empty(T, ng, dtype=torch.float32, device=x.device)
    native().quant_fp8_groups(x, q, s)
    return q, s


def quant_fp8_block_weight(w: torch.Tensor, block: int = 128):
    """Expert weights [E, N, K] -> (e4m3fn, scales [E, ceil(N/128), ceil(K/128)]) per 128x128 block.
    Scales are powers of two: the grouped GEMM hands them to the MFMA as E8M0
    exponents. (Every block-fp8 expert weight of this code base is made here,
    at load and on a weight update; a checkpoint's arbitrary fp32 block scales
    would be re-quantised through this function.)"""
    E, N, K = w.shape
    nb, kb = (N + block - 1) // block, (K + block - 1) // block
    wf = torch.nn.functional.pad(w.float(), (0, kb * block - K, 0, nb * block - N))
    wf = wf.view(E, nb, block, kb, block)
    s = pow2_ceil((wf.abs().amax(dim=(2, 4)) / FP8_MAX).clamp(min=1e-12))
    q = (wf / s[:, :, None, :, None]).clamp(-FP8_MAX, FP8_MAX)
    q = q.view(E, nb * block, kb * block)[:, :N, :K].contiguous().to(FP8)
    return q, s.contiguous()


def _quant_groups_padded(x: torch.Tensor, kp: int, row_limit: Optional[torch.Tensor] = None):
    """quant_fp8_groups into rows of ``kp`` >= d columns, zeros past d, in one kernel (GPU).
    ``row_limit`` (int32 device scalar, e.g. moe_align's padded-slot total): rows at or past it
    are skipped - the grouped GEMM never reads them."""
    T, d = x.shape
    if kp == d and row_limit is None:
        return quant_fp8_groups(x)
    x = x if x.stride(-1) == 1 and x.stride(0) % 8 == 0 else x.contiguous()
    q = torch.empty(T, kp, dtype=FP8, device=x.device)
    s = torch.empty(T, (kp + 127) // 128, dtype=torch.float32, device=x.device)
    native().quant_fp8_groups_padded(x, q, s, row_limit)
    return q, s


def pad_fp8_k(q: torch.Tensor, kp: int) -> torch.Tensor:
    """Zero-pad the K (last) dim of fp8 [..., K] to ``kp`` columns (e4m3 0x00 = +0).
    The v2 grouped GEMM streams whole 128-byte K-steps (one scale block), so
    expert weights whose K is not a multiple of 128 (gpt-oss: 2880) are stored
    padded on the GPU and activations are quantised into padded rows."""
    k = q.shape[-1]
    if kp == k:
        return q
    return torch.nn.functional.pad(q.view(torch.uint8), (0, kp - k)).view(FP8)


def dequant_fp8_block_weight(q: torch.Tensor, s: torch.Tensor, block: int = 128) -> torch.Tensor:
    E, N, K = q.shape
    full = s.repeat_interleave(block, 1).repeat_interleave(block, 2)[:, :N, :K]
    return q.float() * full


# ---------------------------------------------------------------- MXFP4 experts (OCP MX: e2m1 + E8M0 per 32)
_E2M1 = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0)


def quant_mxfp4_weight(w: torch.Tensor):
    """Expert weights [E, N, K] (K % 32 == 0) -> (packed e2m1 codes uint8 [E, N, K / 2]: element 2i in
    the low nibble, 2i + 1 in the high one; E8M0 scales uint8 [E, N, K / 32]) - the OCP MXFP4 format
    gpt-oss ships in. Per 32-element block the scale is the power of two that maps the block's amax
    to <= 6 (the largest e2m1 magnitude); values round to the nearest e2m1 (ties away from zero)."""
    E, N, K = w.shape
    assert K % 32 == 0, "MXFP4 needs K % 32 == 0"
    if E > 1 and w.numel() > (1 << 28):  # keep torch's elementwise grids small: one expert at a time
        parts = [quant_mxfp4_weight(w[e:e + 1]) for e in range(E)]
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
    wf = w.float().contiguous().view(E, N, K // 32, 32)
    amax = wf.abs().amax(-1).clamp(min=2.0 ** -126)
    e = torch.ceil(torch.log2(amax / 6.0)).clamp(-127, 127)
    scale = torch.exp2(e)
    x = (wf / scale[..., None]).clamp(-6.0, 6.0)
    mag = x.abs()
    grid = torch.tensor(_E2M1, device=w.device)
    mids = (grid[1:] + grid[:-1]) / 2
    code = torch.bucketize(mag, mids, right=True).to(torch.uint8)  # ties go up (away from zero)
    code = code | ((x < 0) & (code > 0)).to(torch.uint8) << 3
    code = code.view(E, N, K)
    packed = (code[..., 0::2] | (code[..., 1::2] << 4)).contiguous()
    return packed, (e + 127).to(torch.uint8).contiguous()


def dequant_mxfp4_weight(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """fp32 [E, N, K] of quant_mxfp4_weight's (codes, scales)."""
    E, N, K2 = q.shape
    lo, hi = (q & 0xF).long(), (q >> 4).long()
    codes = torch.stack([lo, hi], -1).view(E, N, 2 * K2)
    grid = torch.tensor(_E2M1, device=q.device)
    v = grid[codes & 7] * torch.where(codes >= 8, -1.0, 1.0)
    scale = torch.exp2(s.float() - 127).repeat_interleave(32, -1)
    return v * scale


def moe_experts_mxfp4(x, ids, wts, w1q, w1s, w2q, w2s, act=0, alpha=1.702, limit=7.0, out=None, b1=None, b2=None):
    """MXFP4 routed experts (gpt-oss's own weight format): e2m1 weights with E8M0 scales per 32
    elements (quant_mxfp4_weight, K padded to 128), activations quantised per (token, 128) group to
    e4m3 with power-of-two scales, both GEMMs on the persistent expert-tile kernel (csrc/ops/moe8.hip
    moe_gemm8_mxfp4_kernel: half the weight bytes of fp8, the scaled MFMA at the fp4 rate) at every
    step size - its weight stream is halved, so it also covers decode-sized steps - and the gated
    activation fused into GEMM 1, bf16 weighted combine. w1q [E, 2F, Kp1/2], w2q [E, d, Kp2/2] in the
    standard packed order (the kernel reads activations in the K order the e2m1 operand implies).
    ``x`` may be ``Fp8Rows`` (the EP dispatch kernel's per-128 e4m3 rows)."""
    E, N1, Kp1 = w1q.shape[0], _mx_n(w1q), _mx_k(w1q)
    d, Kp2 = _mx_n(w2q), _mx_k(w2q)
    F = N1 // 2
    if isinstance(x, Fp8Rows) and not (x.is_cuda and x.q.shape[1] == Kp1):
        x = x.dequant()
    if not isinstance(x, Fp8Rows) and not _gpu(x):
        w1q, w2q = mxfp4_std_layout(w1q), mxfp4_std_layout(w2q)
        w1s, w2s = mxfp4_scales_std_layout(w1s), mxfp4_scales_std_layout(w2s)
        xq, xs = quant_fp8_groups(x)
        xd = (xq.float().view(x.shape[0], -1) * xs.repeat_interleave(128, 1)[:, :x.shape[1]]).to(torch.bfloat16)
        w1 = dequant_mxfp4_weight(w1q, w1s)[..., :x.shape[1]].to(torch.bfloat16)
        w2 = dequant_mxfp4_weight(w2q, w2s)[..., :F].to(torch.bfloat16)
        r = ref.moe_forward(xd, ids, wts, w1, w2, act, alpha, limit, b1, b2)
        if out is not None:
            out.copy_(r)
            return out
        return r
    C = native()
    T = x.shape[0]
    k = ids.shape[1]
    # decode-sized steps: 64-row tiles (4 MFMAs per substep instead of 12-16: the weight stream, not the
    # MFMA work of mostly-empty rows, sets the time)
    bm = 64 if T * k < MXFP4_SMALL_ROWS * E else moe4_tile_rows(T * k, E)
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    dev = x.device
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // bm, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, bm)
    xq, xs = (x.q, x.s) if isinstance(x, Fp8Rows) else _quant_groups_padded(x, Kp1)
    h = torch.empty(max_p, F, dtype=torch.bfloat16, device=dev)
    C.moe_gemm8_mxfp4(xq, xs, k, sorted_ids, tile_e, w1q, w1s, h, 1, act, alpha, limit, False, b1, bm, total)
    hq, hs = _quant_groups_padded(h, Kp2, total)
    y = torch.empty(max_p, d, dtype=torch.bfloat16, device=dev)
    C.moe_gemm8_mxfp4(hq, hs, 1, sorted_ids, tile_e, w2q, w2s, y, 0, 0, 0.0, 0.0, True, b2, bm, total)
    if out is None:
        out = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
    C.moe_combine(y, inv, wts.contiguous().view(-1).float(), k, out)
    return out


# rows per local expert below which the MXFP4 experts take 64-row tiles: with K-step-major weights and
# scales they win at 64 rows (0.548 vs 0.590 ms, gpt-oss layer) and lose at 169 (profiles/moe_mxfp4_r6.txt)
MXFP4_SMALL_ROWS = int(os.environ.get("LLMD_MXFP4_SMALL_ROWS", "72"))


def mxfp4_kernel_layout(q: torch.Tensor) -> torch.Tensor:
    """Packed MXFP4 codes [E, N, K/2] -> K-step major [E, K/128, N, 64]: the 64 code bytes of one
    128-deep K-step of every row of an expert are contiguous, so the tile kernel's weight DMA for a
    K-step of a 256-row tile is one 16 KB run instead of 256 half cache lines (the weight stream is
    most of the kernel's step: profiles/moe_kstep_diag_r6.txt). K % 128 == 0."""
    if q.dim() == 4:
        return q
    E, N, K2 = q.shape
    assert K2 % 64 == 0, "K-step major MXFP4 needs K % 128 == 0"
    return q.view(E, N, K2 // 64, 64).permute(0, 2, 1, 3).contiguous()


def mxfp4_std_layout(q: torch.Tensor) -> torch.Tensor:
    """Inverse of mxfp4_kernel_layout: [E, K/128, N, 64] -> [E, N, K/2] (3-D input unchanged)."""
    if q.dim() == 3:
        return q
    E, nk, N, _ = q.shape
    return q.permute(0, 2, 1, 3).reshape(E, N, nk * 64)


def mxfp4_scales_kernel_layout(s: torch.Tensor) -> torch.Tensor:
    """E8M0 scales [E, N, K/32] -> K-step major [E, K/128, N, 4] (the companion of mxfp4_kernel_layout:
    a K-step's scales of a 256-row tile are one contiguous 1 KB run)."""
    if s.dim() == 4:
        return s
    E, N, nb = s.shape
    return s.view(E, N, nb // 4, 4).permute(0, 2, 1, 3).contiguous()


def mxfp4_scales_std_layout(s: torch.Tensor) -> torch.Tensor:
    if s.dim() == 3:
        return s
    E, nk, N, _ = s.shape
    return s.permute(0, 2, 1, 3).reshape(E, N, nk * 4)


def _mx_n(q):
    return q.shape[2] if q.dim() == 4 else q.shape[1]


def _mx_k(q):
    return 128 * q.shape[1] if q.dim() == 4 else 2 * q.shape[2]


def pad_mxfp4_k(w: torch.Tensor, kp: int) -> torch.Tensor:
    """Zero-pad the K (last) dim of bf16/fp32 expert weights [..., K] to ``kp`` before MXFP4
    quantisation (the tile kernel streams whole 128-deep K-steps)."""
    k = w.shape[-1]
    return w if kp == k else torch.nn.functional.pad(w, (0, kp - k))


# rows per local expert from which the tile GEMMs (v4 bf16 / v8 fp8) replace the 64-row streaming kernels:
# they win from 64 rows on (gpt-oss 1.21-1.25x, DeepSeek EP8 1.29-1.35x) and lose at <= 48
# (profiles/moe_tile_threshold_r6.txt)
MOE_V3_MIN_ROWS = int(os.environ.get("LLMD_MOE_V3_MIN_ROWS", "56"))
MOE_V3 = os.environ.get("LLMD_MOE_V3", "1") == "1"
# bf16 experts on the same 256-row tiles (moe_gemm3 with bf16 operands); LLMD_MOE_V3_BF16=0 keeps v2
MOE_V3_BF16 = os.environ.get("LLMD_MOE_V3_BF16", "1") == "1"  # DeepSeek EP8 T=4096 701 -> 789 TF/s, gpt-oss T=5120 369 -> 529
# bf16 prefill-sized steps on the v4 grouped GEMM (csrc/ops/moe4.hip, the PGR2 structure of the dense
# prefill GEMM): DeepSeek EP8 T=4096 807 -> 1011 TF/s, gpt-oss T=5120 534 -> 586 (profiles/moe_gemm_v4_r5.txt)
MOE_BF16_V4 = os.environ.get("LLMD_MOE_BF16_V4", "1") == "1"
# the persistent form of the v4 bf16 tiles (csrc/ops/moe8.hip moe_gemm8_bf16_kernel): gpt-oss T=5120 layer
# 651 -> 680 TF/s, T=8192 728 -> 748; DeepSeek EP8 (K = 7168 gate/up) 1079 -> 1014, so only GEMMs with
# K <= 4096 take it (profiles/moe_gemm_v8_r6.txt)
MOE_BF16_V8 = os.environ.get("LLMD_MOE_BF16_V8", "1") == "1"
MOE_BF16_V8_MAX_K = int(os.environ.get("LLMD_MOE_BF16_V8_MAX_K", "4096"))
MOE_FUSED_QUANT = os.environ.get("LLMD_MOE_FUSED_QUANT", "0") == "1"
# v4 expert-tile rows: "auto" picks 192 or 256 by the expected padding at T*k/E rows per expert (gpt-oss
# at a 5120-token step: 160 rows -> a 256-row tile is 62 % useful rows, a 192-row one 83 %)
MOE4_TILE = os.environ.get("LLMD_MOE4_TILE", "auto")


def moe4_tile_rows(n_rows: int, E: int) -> int:
    if MOE4_TILE in ("192", "256"):
        return int(MOE4_TILE)
    r = n_rows / max(1, E)
    waste = {t: math.ceil(r / t) * t - r for t in (256, 192)}
    return 192 if waste[192] < waste[256] else 256
# block-fp8 prefill-sized steps on the v4 grouped GEMM (moe4.hip moe_gemm4_fp8_kernel: 4-wave PGR2,
# scaled 32x32x64 MFMA with the E8M0 block scales as operands): DeepSeek EP8 T=4096 1307 -> 1496 TF/s,
# gpt-oss T=5120 757 -> 782 (profiles/moe_gemm_v4_r5.txt)
MOE_FP8_V4 = os.environ.get("LLMD_MOE_FP8_V4", "1") == "1"
# v8: the persistent form of those tiles (csrc/ops/moe8.hip: one workgroup per CU walks XCD-local
# tile chunks, the LDS-DMA stream runs across tile edges, epilogue stored from the accumulators)
# gpt-oss T=5120 gate/up 1053-1069 -> 1175-1191 TF/s, down 993 -> 1140; DeepSeek EP8 T=4096 down 1535 -> 1868
# (profiles/moe_gemm_v8_r6.txt)
MOE_FP8_V8 = os.environ.get("LLMD_MOE_FP8_V8", "1") == "1"
# decode-sized fp8 steps (< MOE_V3_MIN_ROWS rows per expert) on 64-row v8 tiles instead of the 64-row
# weight-streaming kernel (moe.hip moe_gemm_fp8_kernel)
MOE_FP8_T64 = os.environ.get("LLMD_MOE_FP8_T64", "0") == "1"


def moe_tile_version(kind: str, K: int) -> int:
    """Which expert-tile GEMM runs a prefill-sized grouped GEMM of reduction depth K: 8 = the
    persistent form (csrc/ops/moe8.hip; needs >= 4 K-steps: 128-deep fp8, 64-deep bf16), else the
    one-workgroup-per-tile v4 (moe4.hip). bf16 takes v8 only for K <= MOE_BF16_V8_MAX_K: those tiles
    run at the power cap, so hiding the per-tile cost pays only where K-loops are short
    (profiles/moe_gemm_v8_r6.txt)."""
    if kind == "fp8":
        return 8 if MOE_FP8_V8 and K >= 512 else 4
    return 8 if MOE_BF16_V8 and 256 <= K <= MOE_BF16_V8_MAX_K else 4


class Fp8Rows:
    """Activation rows already quantised to block fp8 (e4m3 ``q`` [T, dp] with
    dp = d padded to 128 and zeros past d, fp32 group scales ``s`` [T, dp/128]):
    what the fp8 EP dispatch kernel delivers (parallel/symm.py)."""

    def __init__(self, q: torch.Tensor, s: torch.Tensor, d: int):
        self.q, self.s, self.d = q, s, d

    @property
    def shape(self):
        return torch.Size((self.q.shape[0], self.d))

    @property
    def device(self):
        return self.q.device

    @property
    def is_cuda(self):
        return self.q.is_cuda

    def dequant(self) -> torch.Tensor:
        f = self.q.float() * self.s.repeat_interleave(128, 1)[:, :self.q.shape[1]]
        return f[:, :self.d].to(torch.bfloat16)


def moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act=0, alpha=1.702, limit=7.0, out=None, b1=None, b2=None):
    """Block-scaled FP8 routed experts (DeepGEMM role): activations quantised per
    (token, 128) group, grouped fp8 MFMA GEMMs with 128x128 weight-block scales,
    the gated activation fused into GEMM 1, bf16 weighted combine. ``x`` may be
    ``Fp8Rows`` (quantised by the EP dispatch kernel): no quantisation pass."""
    if isinstance(x, Fp8Rows) and not (x.is_cuda and x.q.shape[1] == w1q.shape[2]):
        x = x.dequant()
    if not isinstance(x, Fp8Rows) and not _gpu(x):
        xq, xs = quant_fp8_groups(x)
        xd = (xq.float().view(x.shape[0], -1) * xs.repeat_interleave(128, 1)[:, :x.shape[1]]).to(torch.bfloat16)
        r = ref.moe_forward(xd, ids, wts, dequant_fp8_block_weight(w1q, w1s).to(torch.bfloat16),
                            dequant_fp8_block_weight(w2q, w2s).to(torch.bfloat16), act, alpha, limit, b1, b2)
        if out is not None:
            out.copy_(r)
            return out
        return r
    C = native()
    T, d = x.shape
    k = ids.shape[1]
    E, N1, Kp1 = w1q.shape
    F = N1 // 2
    Kp2 = w2q.shape[2]
    # prefill-sized steps (>= MOE_V3_MIN_ROWS rows per local expert on average):
    # 256-row expert tiles, one weight pass per expert (moe_gemm3_fp8_kernel);
    # decode-sized steps keep the 64-row weight-streaming kernel
    bm = C.moe_tile_m_prefill() if (T * k >= MOE_V3_MIN_ROWS * E and Kp1 % 128 == 0 and Kp2 % 128 == 0
                                    and MOE_V3) else C.moe_tile_m()
    v4 = (bm == C.moe_tile_m_prefill() and MOE_FP8_V4 and not MOE_FUSED_QUANT and Kp1 <= 8192 and Kp2 <= 8192
          and N1 % 16 == 0 and d % 8 == 0)
    # decode-sized steps on 64-row persistent tiles (moe8.hip, MB = 1) instead of the streaming kernel
    t64 = (not v4 and MOE_FP8_T64 and not MOE_FUSED_QUANT and Kp1 % 128 == 0 and Kp2 % 128 == 0
           and 512 <= min(Kp1, Kp2) and max(Kp1, Kp2) <= 8192 and N1 % 16 == 0 and d % 8 == 0)
    if v4:
        bm = moe4_tile_rows(T * k, E)
    elif t64:
        bm, v4 = 64, True
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    dev = x.device
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // bm, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)  # moe_align fills it (-1 = not on this rank)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, bm)
    if isinstance(x, Fp8Rows):
        xq, xs = x.q, x.s
    else:
        xq, xs = _quant_groups_padded(x, Kp1)
    if MOE_FUSED_QUANT and bm == C.moe_tile_m_prefill() and Kp2 == (N1 + 255) // 256 * 128:
        # 256-row tiles: the first GEMM quantises its activation output itself (opt-in:
        # measured slower - with one workgroup per CU the epilogue's amax exchange and
        # byte stores are not hidden, profiles/moe_gemm_v3_fp8.txt)
        hq = torch.empty(max_p, Kp2, dtype=FP8, device=dev)
        hs = torch.empty(max_p, Kp2 // 128, dtype=torch.float32, device=dev)
        C.moe_gemm_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, torch.empty(0, F, dtype=torch.bfloat16, device=dev),
                       1, act, alpha, limit, False, b1, bm, hq, hs)
    elif v4:
        # v4: PGR2 4-wave tiles, A rows and their act scales gathered by the LDS-DMA (csrc/ops/moe4.hip)
        h = torch.empty(max_p, F, dtype=torch.bfloat16, device=dev)
        v1, v2 = (8, 8) if bm == 64 else (moe_tile_version("fp8", Kp1), moe_tile_version("fp8", Kp2))
        C.moe_gemm4_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, h, 1, act, alpha, limit, False, b1, bm, v1, total)
        hq, hs = _quant_groups_padded(h, Kp2, total)  # slots past the last real tile are never read
        y = torch.empty(max_p, d, dtype=torch.bfloat16, device=dev)
        C.moe_gemm4_fp8(hq, hs, 1, sorted_ids, tile_e, w2q, w2s, y, 0, 0, 0.0, 0.0, True, b2, bm, v2, total)
        if out is None:
            out = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
        C.moe_combine(y, inv, wts.contiguous().view(-1).float(), k, out)
        return out
    else:
        h = torch.empty(max_p, F, dtype=torch.bfloat16, device=dev)
        C.moe_gemm_fp8(xq, xs, k, sorted_ids, tile_e, w1q, w1s, h, 1, act, alpha, limit, False, b1, bm)
        hq, hs = _quant_groups_padded(h, Kp2, total)
    y = torch.empty(max_p, d, dtype=torch.bfloat16, device=dev)
    # second GEMM: A rows are the sorted slots themselves (row p of hq; a_rows_are_slots)
    C.moe_gemm_fp8(hq, hs, 1, sorted_ids, tile_e, w2q, w2s, y, 0, 0, 0.0, 0.0, True, b2, bm)
    if out is None:
        out = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
    C.moe_combine(y, inv, wts.contiguous().view(-1).float(), k, out)
    return out


# ---------------------------------------------------------------- sampling
def sample(logits, temps=None, seeds=None, out_ids=None, want_logprob=False, generator=None):
    if not _gpu(logits):
        ids, lp = ref.sample(logits, temps, generator)
        return ids, (lp if want_logprob else None)
    B = logits.shape[0]
    if out_ids is None:
        out_ids = torch.empty(B, dtype=torch.int64, device=logits.device)
    lp = torch.empty(B, dtype=torch.float32, device=logits.device) if want_logprob else None
    native().sample(logits, temps, seeds, out_ids, lp)
    return out_ids, lp


def topk_topp_mask(logits, topk=None, topp=None, temps=None):
    """In-place top-k then top-p filtering of f32 logits."""
    if not _gpu(logits):
        return ref.topk_topp_mask(logits, topk, topp, temps)
    if topk is not None:
        native().topk_topp_mask(logits, topk, None, temps)
    if topp is not None:
        native().topk_topp_mask(logits, None, topp, temps)
    return logits


rope_cos_sin = ref.rope_cos_sin


# ---------------------------------------------------------------- MoE
def moe_tile_m() -> int:
    return 64


def moe_topk(logits, k, scoring=0, bias=None, n_group=1, topk_group=1, renorm=False, routed_scale=1.0):
    if not _gpu(logits):
        return ref.moe_topk(logits, k, scoring, bias, n_group, topk_group, renorm, routed_scale)
    T = logits.shape[0]
    ids = torch.empty(T, k, dtype=torch.int32, device=logits.device)
    w = torch.empty(T, k, dtype=torch.float32, device=logits.device)
    native().moe_topk(logits.float().contiguous(), k, scoring, bias, n_group, topk_group, renorm,
                      routed_scale, ids, w)
    return ids, w


def moe_experts(x, ids, wts, w1, w2, act=0, alpha=1.702, limit=7.0, out=None, b1=None, b2=None):
    """Fused routed-expert FFN: align -> grouped GEMM (gate_up + gated act) ->
    grouped GEMM (down) -> weighted combine. w1 [E, 2F, d] (interleaved
    gate/up rows), w2 [E, d, F]."""
    if not _gpu(x):
        r = ref.moe_forward(x, ids, wts, w1, w2, act, alpha, limit, b1, b2)
        if out is not None:
            out.copy_(r)
            return out
        return r
    C = native()
    T, d = x.shape
    k = ids.shape[1]
    E, N1, K1 = w1.shape
    F = N1 // 2
    # prefill-sized steps: 256-row expert tiles on the v3 kernel (bf16 form), as moe_experts_fp8
    v3 = T * k >= MOE_V3_MIN_ROWS * E and K1 % 32 == 0 and F % 32 == 0 and MOE_V3 and MOE_V3_BF16
    bm = C.moe_tile_m_prefill() if v3 else C.moe_tile_m()
    v4 = v3 and MOE_BF16_V4 and K1 % 64 == 0 and F % 64 == 0 and N1 % 16 == 0 and d % 8 == 0
    if v4:
        bm = moe4_tile_rows(T * k, E)
    n = T * k
    max_p = ((n + E * (bm - 1)) + bm - 1) // bm * bm
    dev = x.device
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // bm, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)  # moe_align fills it (-1 = not on this rank)
    C.moe_align(ids.contiguous().view(-1), E, sorted_ids, tile_e, offs, total, inv, bm)
    h = torch.empty(max_p, F, dtype=x.dtype, device=dev)
    y = torch.empty(max_p, d, dtype=x.dtype, device=dev)
    if v4:
        # v4: the dense prefill GEMM's 4-wave PGR2 structure, rows gathered by the LDS-DMA (csrc/ops/moe4.hip)
        v1, v2 = moe_tile_version("bf16", w1.shape[2]), moe_tile_version("bf16", w2.shape[2])
        C.moe_gemm4(x, k, sorted_ids, tile_e, w1, h, 1, act, alpha, limit, False, b1, bm, v1, total)
        C.moe_gemm4(h, 1, sorted_ids, tile_e, w2, y, 0, 0, 0.0, 0.0, True, b2, bm, v2, total)
    else:
        C.moe_gemm(x, k, sorted_ids, tile_e, w1, h, 1, act, alpha, limit, False, b1, bm)
        # second GEMM: A rows are the sorted slots themselves (row p of h; a_rows_are_slots)
        C.moe_gemm(h, 1, sorted_ids, tile_e, w2, y, 0, 0, 0.0, 0.0, True, b2, bm)
    if out is None:
        out = torch.empty(T, d, dtype=x.dtype, device=dev)
    C.moe_combine(y, inv, wts.contiguous().view(-1), k, out)
    return out


def mla_split_plan(max_len: int, rows: int, H: int, num_cus: int = 256, fp8: bool = False) -> tuple[int, int]:
    """(split_size, nsplit) so rows x head-groups x splits fills ~2 WGs per CU
    (the v2 kernel runs all 64/128 heads of a row in one workgroup)."""
    v2 = H in (64, 128) and os.environ.get("LLMD_MLA_V1", "0") != "1"
    if v2:
        # one 147 KB-LDS workgroup per CU; a split re-loads the row's 128-head Q
        # (147 KB), so keep >= 4 tiles per split (scripts/bench_mla_split.py sweep:
        # rows 1/8/32/64/128 at ctx 4096 best at 256/256/512/1024/2048 keys)
        groups = 1
        if H == 128:
            try:
                groups = 2 if native().mla_v2_shape(rows, fp8) == 41 else 1
            except (RuntimeError, ImportError, AttributeError):  # no extension (CPU planning)
                groups = 2 if rows <= 16 else 1
        want = max(1, min(math.ceil(max_len / 256), math.ceil(num_cus / max(1, rows * groups))))
        split = max(64, math.ceil(math.ceil(max_len / want) / 64) * 64)
        return split, math.ceil(max(1, max_len) / split)
    base = max(1, rows * ((H + 15) // 16))
    target = 2 * num_cus
    want = max(1, min(math.ceil(max_len / 64), math.ceil(target / base)))
    split = max(64, math.ceil(math.ceil(max_len / want) / 64) * 64)
    return split, math.ceil(max(1, max_len) / split)


def mla_attention(q, cache, block_tables, row_seq, row_len, H, scale, max_len=None, split=None, out=None,
                  workspace=None, kv_scale=1.0, split_dev=None):
    """Absorbed-MLA attention over the paged latent cache (csrc/ops/attn_mla.hip).
    q [R, H*576] bf16, cache [blocks, bs, 576] bf16 or fp8 e4m3fn (dequant
    x kv_scale) -> out [R, H*512]. split_dev: int32 [1] device keys per split
    overriding split[0] (hipGraph replay; nsplit stays the grid)."""
    if not _gpu(q):
        r = ref.mla_attention(q, cache, block_tables, row_seq, row_len, H, scale, kv_scale)
        if out is not None:
            out.copy_(r)
            return out
        return r
    R = q.shape[0]
    if out is None:
        out = torch.empty(R, H * 512, dtype=q.dtype, device=q.device)
    if split is None:
        if max_len is None:
            max_len = int(row_len.max().item()) if R else 1
        split = mla_split_plan(max_len, R, H, fp8=cache.dtype == torch.float8_e4m3fn)
    split_size, nsplit = split
    if nsplit > 1:
        if workspace is None:
            part_o = torch.empty(R * H * nsplit * 512, dtype=torch.float32, device=q.device)
            part_ml = torch.empty(R * H * nsplit * 2, dtype=torch.float32, device=q.device)
        else:
            part_o, part_ml = workspace
    else:
        part_o = part_ml = out.new_empty(0, dtype=torch.float32)
    native().mla_attention(out, q, cache, block_tables, row_seq, row_len, H, scale, split_size, nsplit,
                           part_o, part_ml, kv_scale, split_dev)
    return out


def mla_rope_cache(q, q_lat, kv_c, k_pe, positions, cos_sin, H, slots, cache, kv_scale=1.0):
    """RoPE q_pe into q_lat[..., 512:] and write [kv_c | rope(k_pe)] to the latent
    cache (fp8 e4m3fn caches store saturate(x / kv_scale))."""
    if not _gpu(q):
        return ref.mla_rope_cache(q, q_lat, kv_c, k_pe, positions, cos_sin, H, slots, cache, kv_scale)
    native().mla_rope_cache(q, q_lat, kv_c, k_pe, positions, cos_sin, H, slots, cache, kv_scale)


def lora_bgmv(y, x, A, B, slot, h=None):
    """Multi-LoRA batched GEMV, in place on y (csrc/ops/lora.hip)."""
    if not _gpu(x):
        return ref.lora_bgmv(y, x, A, B, slot)
    if h is None:
        h = torch.empty(x.shape[0] * A.shape[1], dtype=torch.float32, device=x.device)
    native().lora_bgmv(y, x, A, B, slot, h)
    return y


SKINNY_MAX_M = 64
_NUM_CUS = 256
_HBM_BPS = 6.0e12       # sustained streaming rate (MI355X: ~6.3 TB/s for a float4 copy)
_SLOT_BPS = (48e9, 26e9)  # what one workgroup streams at 1 / 2 workgroups per CU


def skinny_plan(M: int, N: int, K: int, num_cus: int = _NUM_CUS) -> tuple[int, int, int]:
    """(rb, nsplit, occ) for the decode GEMM kernel (csrc/ops/skinny_gemm.hip):
    rb row blocks of 16 W rows per workgroup, nsplit-way split-K, occ workgroups
    per CU. Cost model: W (HBM) + X (L2, a quarter of the price) bytes per
    workgroup over its streaming rate, times the dispatch rounds, plus the
    split-K partial round trip and the reduce launch."""
    key = ((M + 15) // 16, N, K)
    if key in SKINNY_TUNED:
        return SKINNY_TUNED[key]
    nat = native()
    best, best_t = None, float("inf")
    nq = K // 256
    for occ in (2, 1):
        slots = num_cus * occ
        for rb in range(1, 9):
            if not nat.skinny_supported(M, rb, occ):
                continue
            tiles = -(-N // (16 * rb))
            for ns in range(1, min(nq, 32) + 1):
                per = -(-nq // ns)
                ns2 = -(-nq // per)
                wgs = tiles * ns2
                rounds = -(-wgs // slots)
                busy = min(wgs, slots)
                rate = min(_SLOT_BPS[occ - 1], _HBM_BPS / busy)
                wbytes = 16 * rb * per * 256 * 2
                xbytes = M * per * 256 * 2
                t = rounds * (wbytes + 0.25 * xbytes) / rate
                if ns2 > 1:
                    t += 2.5e-6 + ns2 * M * N * 8 / 8e12
                if t < best_t - 1e-9:
                    best, best_t = (rb, ns2, occ), t
    return best


# measured best plans (scripts/bench_gemm.py --sweep): (ceil(M/16), N, K) -> (rb, nsplit, occ)
SKINNY_TUNED: dict[tuple[int, int, int], tuple[int, int, int]] = {}


def skinny_gemm(x: torch.Tensor, w: torch.Tensor, plan: Optional[tuple[int, int, int]] = None) -> torch.Tensor:
    M, K = x.shape
    N = w.shape[0]
    rb, ns, occ = plan or skinny_plan(M, N, K)
    y = torch.empty(M, N, dtype=x.dtype, device=x.device)
    part = torch.empty(ns * M * N if ns > 1 else 0, dtype=torch.float32, device=x.device)
    native().skinny_gemm(y, x, w, rb, ns, occ, part)
    return y


def skinny_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    M = x.shape[0] if x.dim() == 2 else -1
    return (_gpu(x) and 1 <= M <= SKINNY_MAX_M and x.shape[1] % 256 == 0 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.shape[0] % 4 == 0 and x.stride(-1) == 1 and x.stride(0) % 8 == 0
            and w.is_contiguous())


_DGEMM_MS = (1, 8, 16, 32, 48, 64)


def dgemm_choice(M: int, N: int, K: int) -> Optional[tuple[int, int, int]]:
    """Plan of the decode GEMM kernel for this shape, or None for hipBLASLt:
    the measured dispatch table (ops/dgemm_table.py) at the smallest measured
    M >= this one; unmeasured shapes stay on hipBLASLt."""
    from .dgemm_table import DGEMM_TABLE

    for m in _DGEMM_MS:
        if m >= M:
            e = DGEMM_TABLE.get((m, N, K))
            return e[0] if e is not None else None
    return None


def mgemm(x: torch.Tensor, w: torch.Tensor, plan: tuple[int, int, int]) -> torch.Tensor:
    """Y = X W^T for 33 <= M <= 256 on the LDS-DMA medium-M decode GEMM
    (csrc/ops/mgemm.hip); plan = (wrb: 64-row W tiles per workgroup, nsplit,
    stages)."""
    M, K = x.shape
    N = w.shape[0]
    wrb, ns, stages = plan
    y = torch.empty(M, N, dtype=x.dtype, device=x.device)
    part = torch.empty(ns * M * N if ns > 1 else 0, dtype=torch.float32, device=x.device)
    native().mgemm(y, x, w, wrb, ns, stages, part)
    return y


# decode o / down projection with the following residual-add + RMSNorm in the medium-M GEMM's split-K
# reduce (LLMD_MGEMM_NORM=0: the plain GEMM + reduce + fused_add_rms_norm kernels)
MGEMM_NORM = os.environ.get("LLMD_MGEMM_NORM", "1") == "1"


def mgemm_norm_plan(x: torch.Tensor, w: torch.Tensor) -> Optional[tuple[int, int, int]]:
    """The shipped medium-M plan of this projection when it is split over K (so its partials can be
    reduced together with the residual-add + RMSNorm), else None."""
    if not (MGEMM_NORM and _SKINNY and x.dim() == 2 and 33 <= x.shape[0] <= 128 and mgemm_ok(x, w)
            and w.shape[0] % 8 == 0 and w.shape[0] <= 8192 and w.shape[1] >= 128):
        return None
    plan = mgemm_choice(x.shape[0], w.shape[0], w.shape[1])
    if plan is None or plan[1] < 2:
        return None
    return plan


def mgemm_partials(x: torch.Tensor, w: torch.Tensor, plan: tuple[int, int, int]):
    """Split-K partials of x W^T on the medium-M GEMM, for a consumer that fuses the reduce:
    returns (fp32 partials [nsplit * M * N], nsplit)."""
    M, N = x.shape[0], w.shape[0]
    part = torch.empty(plan[1] * M * N, dtype=torch.float32, device=x.device)
    ns = native().mgemm_partials(x, w, plan[0], plan[1], plan[2], part)
    return part, int(ns)


def reduce_rope_cache(part: torch.Tensor, nsplit: int, qkv: torch.Tensor, positions, cos_sin, Hq, Hkv, D, slots,
                      k_cache, v_cache, neox=True, k_scale=1.0, v_scale=1.0):
    """The QKV projection's split-K reduce + RoPE + paged KV write in one kernel (rope_cache.hip):
    ``qkv`` [T, W] (allocated, unwritten) receives the projection with Q rotated - bit-identical to
    mgemm + rope_cache."""
    native().reduce_rope_cache(part, nsplit, qkv, positions, cos_sin, Hq, Hkv, D, slots, k_cache, v_cache, neox,
                               k_scale, v_scale)


def mgemm_add_rmsnorm(x: torch.Tensor, w: torch.Tensor, plan: tuple[int, int, int], residual: torch.Tensor,
                      gamma: torch.Tensor, eps: float) -> torch.Tensor:
    """residual += x W^T (rounded to bf16); returns rmsnorm(residual) * gamma - bit-identical to
    ``linear`` + ``fused_add_rms_norm`` (csrc/ops/mgemm.hip mgemm_reduce_norm_kernel)."""
    M, N = x.shape[0], w.shape[0]
    wrb, ns, stages = plan
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    part = torch.empty(ns * M * N, dtype=torch.float32, device=x.device)
    native().mgemm_add_rmsnorm(out, x, w, wrb, ns, stages, part, residual, gamma, eps)
    return out


# decode gate/up projection with the SiLU-and-mul in the medium-M GEMM's epilogue (LLMD_MGEMM_SILU=0:
# the plain GEMM + act kernel)
MGEMM_SILU = os.environ.get("LLMD_MGEMM_SILU", "1") == "1"


def mgemm_silu_plan(x: torch.Tensor, w: torch.Tensor) -> Optional[tuple[int, int, int]]:
    """The shipped medium-M plan of the [gate; up] GEMM when it runs whole-K tiles of 2 or 4
    W row blocks (the fused form's shape), else None."""
    if not (MGEMM_SILU and x.dim() == 2 and 33 <= x.shape[0] <= 256 and mgemm_ok(x, w) and w.shape[0] % 8 == 0):
        return None
    plan = mgemm_choice(x.shape[0], w.shape[0], w.shape[1])
    if plan is None or plan[1] != 1 or plan[0] not in (2, 4):
        return None
    if x.shape[0] > 128 and (plan[0], plan[2]) != (2, 3):  # the only ACT form of the 192 / 256-row tiles
        return None
    return plan


def mgemm_silu(x: torch.Tensor, w: torch.Tensor, plan: tuple[int, int, int]) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) for w = [gate; up] [2F, K], M 33..256 (csrc/ops/mgemm.hip ACT form)."""
    y = torch.empty(x.shape[0], w.shape[0] // 2, dtype=x.dtype, device=x.device)
    native().mgemm_silu(y, x, w, plan[0], plan[2])
    return y


def mgemm_fp8(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
              plan: tuple[int, int, int]) -> torch.Tensor:
    """Y = (Xq sx)(Wq sw)^T on the medium-M GEMM's fp8 form (e4m3fn operands, per-token
    scales xs [M, 1], per-channel scales ws [1, N]; K % 128 == 0), bf16 out."""
    M = xq.shape[0]
    N = wq.shape[0]
    wrb, ns, stages = plan
    y = torch.empty(M, N, dtype=torch.bfloat16, device=xq.device)
    part = torch.empty(ns * M * N if ns > 1 else 0, dtype=torch.float32, device=xq.device)
    native().mgemm_fp8(y, xq, xs, wq, ws, wrb, ns, stages, part)
    return y


def mgemm_fp8_choice(M: int, N: int, K: int) -> Optional[tuple[int, int, int]]:
    """Plan of the fp8 medium-M GEMM for this shape (ops/mgemm_fp8_table.py,
    winners over hipBLASLt's tuned scaled GEMM) at the smallest measured M >= M."""
    from .mgemm_fp8_table import MGEMM_FP8_TABLE

    if M < 33 or K % 128:
        return None
    for m in _MGEMM_MS:
        if m >= M:
            e = MGEMM_FP8_TABLE.get((m, N, K))
            return e[0] if e is not None else None
    return None


def mgemm_ok(x: torch.Tensor, w: torch.Tensor, max_m: int = 256) -> bool:
    """Shapes the medium-M kernel takes (plain / fp8 / SiLU forms up to 256 rows; the forms with a
    fused split-K reduce pass max_m=128)."""
    M = x.shape[0] if x.dim() == 2 else -1
    return (_gpu(x) and 1 <= M <= max_m and x.shape[1] % 64 == 0 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.shape[0] % 4 == 0 and x.stride(-1) == 1 and x.stride(0) % 8 == 0
            and w.is_contiguous())


_MGEMM_MS = (64, 96, 128, 192, 256)


PGEMM_VARIANT = int(os.environ.get("LLMD_PGEMM_VARIANT", "0"))


def pgemm(x: torch.Tensor, w: torch.Tensor, epi: int = 0, out: Optional[torch.Tensor] = None,
          variant: Optional[int] = None, split_k: bool = True) -> torch.Tensor:
    """Y = X W^T on the prefill GEMM (csrc/ops/pgemm.hip: 256 x 256 LDS-DMA MFMA
    tiles; N % 256 == 0, K % 64 == 0, any M). epi=1: ``w`` holds gate/up rows
    interleaved per 256-row tile (pgemm_pack_gate_up) and the kernel stores
    silu(gate) * up, [M, N / 2]. ``split_k`` (variant 1, epi 0): a last wave of
    tiles at most half full runs split over K (fp32 partials + reduce)."""
    M = x.shape[0]
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N // 2 if epi in (1, 3) else N, dtype=x.dtype, device=x.device)
    native().pgemm(out, x, w, epi, PGEMM_VARIANT if variant is None else variant, split_k)
    return out


def pgemm_silu(x: torch.Tensor, w: torch.Tensor, variant: int = 3, out: Optional[torch.Tensor] = None):
    """silu(x W_gate^T) * (x W_up^T) in ONE prefill GEMM on the model's own fused [gate; up]
    weight ([2F, K], F % 128 == 0): each 256-column tile loads 128 gate rows and the matching
    128 up rows, the epilogue stores the activation [M, F] (no [M, 2F] round trip, no act kernel)."""
    return pgemm(x, w, epi=3, out=out, variant=variant, split_k=False)


def pgemm_pack_gate_up(w: torch.Tensor) -> torch.Tensor:
    """[2F, K] (gate rows, then up rows) -> the fused-SiLU pgemm layout: per
    256-row tile, 128 gate rows then the matching 128 up rows (F % 128 == 0)."""
    F2, K = w.shape
    F = F2 // 2
    assert F % 128 == 0, F
    g = w[:F].view(F // 128, 128, K)
    u = w[F:].view(F // 128, 128, K)
    return torch.stack((g, u), 1).reshape(F2, K).contiguous()


def pgemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.is_cuda
            and w.shape[0] % 256 == 0 and w.shape[1] % 64 == 0 and x.stride(-1) == 1 and x.stride(0) % 8 == 0
            and w.is_contiguous())


def mgemm_choice(M: int, N: int, K: int) -> Optional[tuple[int, int, int]]:
    """Plan of the medium-M decode GEMM for this shape, or None: the measured
    table (ops/mgemm_table.py, winners over hipBLASLt and the small-M kernel)
    at the smallest measured M >= this one."""
    from .mgemm_table import MGEMM_TABLE

    for m in _MGEMM_MS:
        if m >= M:
            e = MGEMM_TABLE.get((m, N, K))
            return e[0] if e is not None else None
    return None


# Prefill-sized GEMMs: the hand-written prefill GEMM (pgemm) where it beats hipBLASLt ON THIS
# SHAPE. The choice is a STATIC table measured offline (ops/pgemm_table.py, written by
# scripts/make_pgemm_table.py): keyed by (M bucket of 256 rows, N, K), so every run and every
# TP / EP rank picks the same kernel and no forward ever stalls on a timing run.
# LLMD_PGEMM_AUTO=measure restores the old first-sight timing (tuning only); =0 disables pgemm.
PGEMM_AUTO = os.environ.get("LLMD_PGEMM_AUTO", "table")
PGEMM_MIN_M = int(os.environ.get("LLMD_PGEMM_MIN_M", "256"))
_pgemm_pick: dict = {}


def _time_ms(fn, reps: int = 2) -> float:
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps


def pgemm_plan(M: int, N: int, K: int) -> Optional[tuple[int, bool]]:
    """(variant, split_k) of the prefill GEMM for this shape from the shipped table, or None
    (hipBLASLt)."""
    from .pgemm_table import PGEMM_TABLE

    e = PGEMM_TABLE.get(((M + 255) // 256, N, K))
    return None if e is None else e[0]


def pgemm_silu_plan(x: torch.Tensor, w: torch.Tensor) -> Optional[int]:
    """Variant of the fused gate/up + SiLU prefill GEMM (pgemm_silu) for this shape from the
    shipped table (entries keyed ("silu", M bucket, N, K)), or None: hipBLASLt + act kernel."""
    if PGEMM_AUTO == "0" or x.shape[0] < PGEMM_MIN_M or not pgemm_ok(x, w) or (w.shape[0] // 2) % 128:
        return None
    from .pgemm_table import PGEMM_TABLE

    e = PGEMM_TABLE.get(("silu", (x.shape[0] + 255) // 256, w.shape[0], w.shape[1]))
    return None if e is None or e[0] is None else e[0][0]


def pgemm_wins(x: torch.Tensor, w: torch.Tensor) -> Optional[tuple[int, bool]]:
    """The pgemm plan for this GEMM, or None for hipBLASLt."""
    M, (N, K) = x.shape[0], w.shape
    if PGEMM_AUTO != "measure":
        return pgemm_plan(M, N, K)
    key = ((M + 255) // 256, N, K)
    c = _pgemm_pick.get(key, False)
    if c is False:
        if torch.cuda.is_current_stream_capturing():
            return None
        y = torch.empty(M, N, dtype=x.dtype, device=x.device)
        t_pg = _time_ms(lambda: pgemm(x, w, out=y))
        t_bl = _time_ms(lambda: torch.nn.functional.linear(x, w))
        c = _pgemm_pick[key] = (PGEMM_VARIANT, True) if t_pg < 0.97 * t_bl else None
        msg = (f"prefill GEMM M~{M} N={N} K={K}: pgemm {t_pg:.3f} ms, hipBLASLt {t_bl:.3f} ms -> "
               f"{'pgemm' if c else 'hipBLASLt'}")
        log.debug(msg)
        if os.environ.get("LLMD_PGEMM_VERBOSE") == "1":
            import sys

            print(msg, file=sys.stderr, flush=True)
    return c


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Dense projection: decode-sized M on our decode GEMM kernels where their
    measured dispatch tables have them ahead of hipBLASLt - the medium-M LDS-DMA
    kernel (csrc/ops/mgemm.hip, M 33..128, ops/mgemm_table.py) first, then the
    stream kernel (csrc/ops/skinny_gemm.hip, M <= 64, ops/dgemm_table.py) -
    prefill-sized M on the prefill GEMM where the shipped table (ops/pgemm_table.py)
    has it ahead of hipBLASLt - everything else on hipBLASLt."""
    if PGEMM_AUTO != "0" and x.dim() == 2 and x.shape[0] >= PGEMM_MIN_M and pgemm_ok(x, w):
        plan = pgemm_wins(x, w)
        if plan is not None:
            y = pgemm(x, w, variant=plan[0], split_k=plan[1])
            return y if bias is None else y.add_(bias)
    if _SKINNY:
        M = x.shape[0] if x.dim() == 2 else 0
        if 33 <= M <= 256 and mgemm_ok(x, w):
            plan = mgemm_choice(M, w.shape[0], w.shape[1])
            if plan is not None:
                y = mgemm(x, w, plan)
                return y if bias is None else y.add_(bias)
        if skinny_ok(x, w):
            plan = dgemm_choice(M, w.shape[0], w.shape[1])
            if plan is not None:
                y = skinny_gemm(x, w, plan)
                return y if bias is None else y.add_(bias)
    return torch.nn.functional.linear(x, w, bias)


_SKINNY = os.environ.get("LLMD_SKINNY_GEMM", "1") == "1"
