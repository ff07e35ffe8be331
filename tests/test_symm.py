"""Symmetric IPC heap: custom all-reduce + wide-EP low-latency dispatch/combine.

GPU: scripts/symm_check.py with 2 and 4 processes sharing cuda:0 (hipIpc
between processes, per-workgroup epoch barriers, graph replays) against fp32
references. CPU: backend selection / layout arithmetic.
"""
import json
import os
import subprocess
import sys

import pytest

from llmd_amd.parallel import ep, symm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_backend_aliases():
    assert ep.canonical("deepep_low_latency") == "symm_ll"
    assert ep.canonical("deepep_high_throughput") == "symm_ht"
    ep.set_backend("deepep_low_latency")
    assert ep.backend() == "symm_ll"
    ep.set_backend("allgather_reducescatter")
    with pytest.raises(ValueError):
        ep.set_backend("nvshmem")


def test_ht_chunk_plan():
    assert ep.chunk_plan(4096, 1024) == (4, 1024)
    assert ep.chunk_plan(1025, 1024) == (2, 513)
    assert ep.chunk_plan(10, 1024) == (1, 10)
    for R in range(1, 3000, 37):
        n, rc = ep.chunk_plan(R, 256)
        assert rc <= 256 and n * rc >= R and (n - 1) * rc < R


def test_ep_heap_bytes_cover_layout():
    # the layout carved by SymmEP must fit in heap_bytes for any world size
    for world in (1, 2, 8):
        for rows, d, k in ((256, 7168, 8), (64, 2880, 4), (96, 256, 4)):
            need = symm.SymmEP.heap_bytes(world, rows, d, k)
            rx = world * rows * d * 2
            rid = world * rows * k * 4
            assert need >= 2 * rx + 2 * rid


class _FakeHeap:
    """SymmHeap stand-in on the CPU: a byte tensor carved like the real one."""

    def __init__(self, nbytes, world):
        import torch

        self.world, self.rank = world, 0
        self.heap = torch.full((nbytes,), 0xAB, dtype=torch.uint8)
        self._next = 4096
        self.nbytes = nbytes

    carve = symm.SymmHeap.carve


@pytest.mark.parametrize("world,rows,d,k", [(1, 16, 320, 4), (8, 256, 7168, 8), (4, 64, 2880, 4)])
def test_ep_fp8_layout_fits_and_views(world, rows, d, k):
    import torch

    need = symm.SymmEP.heap_bytes(world, rows, d, k, fp8=True)
    h = _FakeHeap(need + 4096, world)
    sep = symm.SymmEP(h, rows, d, k, fp8=True)
    lay = sep.layout
    assert len(lay) == 7 and lay[5] > lay[3] and lay[6] > lay[5]
    dp = (d + 127) // 128 * 128
    assert lay[6] + world * rows * (dp // 128) * 4 <= h.nbytes
    rx, rid, rw = sep.views(rows)
    assert rx.q.dtype == torch.float8_e4m3fn and tuple(rx.q.shape) == (world * rows, dp)
    assert tuple(rx.s.shape) == (world * rows, dp // 128) and tuple(rx.shape) == (world * rows, d)
    assert bool((rx.q.view(torch.uint8) == 0).all())  # padding zeroed at construction
    # bf16 layouts keep the fp8 areas disabled
    h2 = _FakeHeap(symm.SymmEP.heap_bytes(world, rows, d, k) + 4096, world)
    assert symm.SymmEP(h2, rows, d, k).layout[5:] == [-1, -1]


def test_fp8_rows_dequant_feeds_bf16_experts():
    import torch

    from llmd_amd import ops

    x = torch.randn(5, 200).to(torch.bfloat16)
    q, s = ops.quant_fp8_groups(x)
    q = torch.nn.functional.pad(q.view(torch.uint8), (0, 56)).view(torch.float8_e4m3fn)
    r = ops.Fp8Rows(q, s, 200)
    assert tuple(r.shape) == (5, 200)
    dq = r.dequant()
    assert dq.shape == (5, 200)
    assert (dq.float() - x.float()).abs().max() <= x.float().abs().max() / 8


def test_symm_ll_falls_back_on_cpu():
    """On CPU tensors the symm backend must take the RCCL/gloo path (no heap)."""
    import torch

    from llmd_amd.parallel.state import ParallelState, get_state, set_state

    old = get_state()
    set_state(ParallelState())  # world 1: moe_ep collectives degenerate
    try:
        ep.set_backend("symm_ll")
        x = torch.randn(3, 8)
        ids = torch.tensor([[0, 1], [1, -1], [0, 0]], dtype=torch.int32)
        w = torch.ones(3, 2)
        calls = []

        def fn(xx, ii, ww):
            calls.append(ii.clone())
            return xx * 2

        ep.set_step_rows(0)
        import torch.distributed as dist

        if not dist.is_initialized():
            # world-1 gloo group so the fallback collectives run
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29633")
            dist.init_process_group("gloo", rank=0, world_size=1)
            st = ParallelState(world_size=1, ep_group=dist.group.WORLD, cpu_group=dist.group.WORLD)
            set_state(st)
            try:
                y = ep.moe_ep(x, ids, w, 2, fn)
            finally:
                dist.destroy_process_group()
            assert torch.allclose(y, x * 2)
            assert calls
    finally:
        ep.set_backend("allgather_reducescatter")
        set_state(old)


def _run(nproc, port, extra_env=None):
    env = dict(os.environ, LLMD_SYMM_DEVICE="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "scripts", "symm_check.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["ok"] and d["timeout_flag"] == 0
    return d


@pytest.mark.gpu
def test_symm_collectives_2proc():
    d = _run(2, 29641)
    assert d["world"] == 2


@pytest.mark.gpu
def test_symm_collectives_4proc():
    d = _run(4, 29642)
    assert d["world"] == 4
