"""Expert-parallel token exchange for wide-EP (DP attention + EP MoE; SURVEY
K12, M03-M06; reference guides/wide-ep-lws, `--all2all-backend`).

Each rank owns E / EP experts and its own tokens. Two exchange backends:

* ``allgather_reducescatter`` (default, the reference's single-node
  fallback): all-gather every rank's tokens + routing (equal row counts:
  rows are padded to the step's max, agreed by the DP coordinator), run the
  local experts on all rows, reduce-scatter the partial outputs back. Fixed
  shapes -> hipGraph-capturable decode.
* ``alltoall`` (DeepEP role): every token is sent once to each rank that owns
  at least one of its top-k experts, carrying the per-rank (local expert,
  weight) list; RCCL ``all_to_all_single`` with variable splits dispatches,
  the local grouped GEMM runs on exactly the received rows, a second
  all-to-all returns the weighted partial outputs, which are summed per token.
  Moves ~(distinct ranks per token)/EP of the all-gather volume; needs the
  split sizes on the host (one small count exchange per layer), so eager only.

* ``symm_ll`` (alias ``deepep_low_latency``): the HIP dispatch/combine
  kernels over the symmetric IPC heap (parallel/symm.py) for steps of at most
  the heap's row capacity: each token row is pushed straight into the
  owning ranks' receive buffers over xGMI (7 links at once), fixed shapes, so
  decode graphs capture it.
* ``symm_ht`` (alias ``deepep_high_throughput``): prefill-sized steps through
  the same kernels in chunks of the heap's row capacity. The chunk count comes
  from the step's agreed max rows (DP coordinator), so no per-layer count
  exchange or host sync is needed (the RCCL ``alltoall`` backend needs
  ``.tolist()`` of the split sizes), the exchange stays on the GPU and the
  whole prefill MoE is graph-capturable. Each chunk's grouped GEMM still sees
  world x chunk rows. Without a heap (CPU, multi-node) it degrades to
  ``alltoall``.

``expert_fn(x, local_ids, weights) -> y`` computes the weighted sum over the
given local experts (-1 ids are skipped).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .state import get_state

BACKENDS = ("allgather_reducescatter", "alltoall", "symm_ll", "symm_ht")
ALIASES = {"deepep_low_latency": "symm_ll", "deepep_high_throughput": "symm_ht"}
_backend = "allgather_reducescatter"
_step_rows = 0  # max token rows of this step over the EP group (DP coordinator)


def canonical(name: str) -> str:
    return ALIASES.get(name, name)


def set_backend(name: str):
    global _backend
    name = canonical(name)
    if name not in BACKENDS:
        raise ValueError(f"all2all backend must be one of {BACKENDS}")
    _backend = name


def backend() -> str:
    return _backend


def set_step_rows(n: int):
    global _step_rows
    _step_rows = int(n)


def ep_active() -> bool:
    st = get_state()
    return st.dp_size > 1 and st.tp_size == 1


def moe_ep(x: torch.Tensor, ids: torch.Tensor, w: torch.Tensor, E_local: int, expert_fn) -> torch.Tensor:
    capturing = x.is_cuda and torch.cuda.is_current_stream_capturing()
    if _backend in ("symm_ll", "symm_ht") and x.is_cuda:
        from . import symm

        sep = symm.ep()
        R = max(x.shape[0], _step_rows)
        if sep is not None and R <= sep.R_max:
            return sep.moe(x, ids, w, E_local, R, expert_fn)
        if sep is not None and _step_rows >= x.shape[0]:
            # the chunk count must agree over the EP group: only from the agreed step rows
            return symm_chunked(sep, x, ids, w, E_local, _step_rows, expert_fn)
    if _backend in ("alltoall", "symm_ll", "symm_ht") and not capturing:
        return _alltoall(x, ids, w, E_local, expert_fn)
    return _allgather(x, ids, w, E_local, expert_fn)


def chunk_plan(R: int, cap: int) -> tuple[int, int]:
    """(chunks, rows per chunk) covering R rows with chunks of at most ``cap``,
    balanced so the last chunk is not nearly empty."""
    n = -(-R // cap)
    return n, -(-R // n)


def symm_chunked(sep, x, ids, w, E_local, R, expert_fn):
    """HT exchange: ``R`` (agreed over the group) rows in equal chunks through
    the symm dispatch/combine kernels; ranks whose own rows run out still take
    part in every chunk with empty slices."""
    T = x.shape[0]
    n, rc = chunk_plan(R, sep.R_max)
    outs = []
    for c in range(n):
        a, b = min(c * rc, T), min((c + 1) * rc, T)
        outs.append(sep.moe(x[a:b], ids[a:b], w[a:b], E_local, rc, expert_fn))
    return torch.cat(outs) if len(outs) > 1 else outs[0]


def _allgather(x, ids, w, E_local, expert_fn):
    st = get_state()
    T = x.shape[0]
    rows = max(T, _step_rows)
    if rows > T:  # pad to the step's max rows: collectives need equal shapes
        x = torch.cat([x, x.new_zeros(rows - T, x.shape[1])])
        ids = torch.cat([ids, ids.new_full((rows - T, ids.shape[1]), -1)])
        w = torch.cat([w, w.new_zeros(rows - T, w.shape[1])])
    g = st.ep_group
    n = st.ep_size
    xs = torch.empty((n * rows, x.shape[1]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(xs, x.contiguous(), group=g)
    ia = torch.empty((n * rows, ids.shape[1]), dtype=ids.dtype, device=ids.device)
    dist.all_gather_into_tensor(ia, ids.contiguous(), group=g)
    wa = torch.empty((n * rows, w.shape[1]), dtype=w.dtype, device=w.device)
    dist.all_gather_into_tensor(wa, w.contiguous(), group=g)
    lo = st.ep_rank * E_local
    local = (ia >= lo) & (ia < lo + E_local)
    y = expert_fn(xs, torch.where(local, ia - lo, torch.full_like(ia, -1)), torch.where(local, wa, 0.0))
    out = torch.empty((rows, y.shape[1]), dtype=y.dtype, device=y.device)
    dist.reduce_scatter_tensor(out, y.contiguous(), group=g)
    return out[:T]


def _alltoall(x, ids, w, E_local, expert_fn):
    st = get_state()
    g, n = st.ep_group, st.ep_size
    T, k = ids.shape
    dev = x.device
    dest = torch.where(ids >= 0, ids // E_local, torch.full_like(ids, n))        # [T, k] owner rank
    # one message per (token, destination rank)
    onehot = torch.zeros(T, n + 1, dtype=torch.bool, device=dev)
    onehot.scatter_(1, dest.long(), True)
    onehot = onehot[:, :n]
    tok, rnk = onehot.nonzero(as_tuple=True)                                      # sorted by token
    order = torch.argsort(rnk, stable=True)
    tok, rnk = tok[order], rnk[order]                                             # grouped by rank
    send_counts = torch.bincount(rnk, minlength=n)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=g)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    # per message: the token row and its k (local id | -1, weight) for that rank
    sel = dest[tok] == rnk[:, None]                                               # [M, k]
    lid = torch.where(sel, ids[tok] - rnk[:, None] * E_local, torch.full_like(ids[tok], -1))
    lw = torch.where(sel, w[tok], torch.zeros_like(w[tok]))
    M_in = sum(rc)
    x_recv = torch.empty((M_in, x.shape[1]), dtype=x.dtype, device=dev)
    dist.all_to_all_single(x_recv, x[tok].contiguous(), rc, sc, group=g)
    id_recv = torch.empty((M_in, k), dtype=lid.dtype, device=dev)
    dist.all_to_all_single(id_recv, lid.contiguous(), rc, sc, group=g)
    w_recv = torch.empty((M_in, k), dtype=lw.dtype, device=dev)
    dist.all_to_all_single(w_recv, lw.contiguous(), rc, sc, group=g)
    y_recv = expert_fn(x_recv, id_recv, w_recv) if M_in else x_recv.new_zeros(0, x.shape[1])
    y_back = torch.empty((len(tok), y_recv.shape[1]), dtype=y_recv.dtype, device=dev)
    dist.all_to_all_single(y_back, y_recv.contiguous(), sc, rc, group=g)
    out = torch.zeros((T, y_back.shape[1]), dtype=torch.float32, device=dev)
    out.index_add_(0, tok, y_back.float())
    return out.to(x.dtype)
