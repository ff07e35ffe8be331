"""Measure the prefill GEMM choice offline and write llmd_amd/ops/pgemm_table.py.

For every (M bucket of 256 rows, N, K) of the served models' prefill
projections, time hipBLASLt (F.linear) against the hand-written pgemm variants
(with and without the split-K tail) on random [-1, 1) operands, interleaved
rounds in one process, and keep a pgemm plan only where it beats hipBLASLt by
>= --margin. The engine then picks by table lookup - the same choice on every
run and every TP / EP rank, no timing inside a forward.

  python scripts/make_pgemm_table.py [--rounds 3] [--variants 0,3] [--out llmd_amd/ops/pgemm_table.py]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402

# (N, K) of the prefill projections: Llama-3-70B TP1 / TP2 / TP4 shards, Llama-3-8B TP1, Qwen3-32B TP1
SHAPES = {
    "70b": [(10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672)],
    "70b_tp2": [(5120, 8192), (8192, 4096), (28672, 8192), (8192, 14336)],
    "70b_tp4": [(2560, 8192), (8192, 2048), (14336, 8192), (8192, 7168)],
    "8b": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)],
    "32b": [(10240, 5120), (5120, 8192), (51200, 5120), (5120, 25600)],
}
BUCKETS = (2, 3, 4, 6, 8, 12, 16, 18, 20, 24, 32)
GATE_UP = {57344, 28672, 14336, 51200}  # fused [gate; up] widths (2F) of the served models


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,3")
    ap.add_argument("--models", default=",".join(SHAPES))
    ap.add_argument("--buckets", default=",".join(map(str, BUCKETS)))
    ap.add_argument("--margin", type=float, default=0.03)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "llmd_amd", "ops", "pgemm_table.py"))
    a = ap.parse_args()
    vs = [int(v) for v in a.variants.split(",")]
    shapes = sorted({s for m in a.models.split(",") for s in SHAPES[m]})
    buckets = [int(b) for b in a.buckets.split(",")]
    torch.manual_seed(0)
    rows = []
    t_start = time.time()
    for N, K in shapes:
        w = torch.rand(N, K, device="cuda").mul_(2).sub_(1).to(torch.bfloat16)
        for mb in buckets:
            M = mb * 256 - 128 if mb > 2 else mb * 256 - 6  # a bucket's typical (non-aligned) size
            x = torch.rand(M, K, device="cuda").mul_(2).sub_(1).to(torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            it = max(3, int(1e13 / (2.0 * M * N * K)))
            cands = {"blas": lambda: F.linear(x, w)}
            for v in vs:
                cands[(v, False)] = (lambda v=v: ops.pgemm(x, w, out=y, variant=v, split_k=False))
                cands[(v, True)] = (lambda v=v: ops.pgemm(x, w, out=y, variant=v, split_k=True))
            res = {k: [] for k in cands}
            for _ in range(a.rounds):
                for k, fn in cands.items():
                    res[k].append(timeit(fn, it))
            med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
            best = min((k for k in med if k != "blas"), key=lambda k: med[k])
            pick = best if med[best] < (1 - a.margin) * med["blas"] else None
            rows.append((mb, N, K, pick, med[best] * 1e3, med["blas"] * 1e3))
            print(f"M~{M:5d} (bucket {mb:2d}) N={N:6d} K={K:6d}: blas {med['blas'] * 1e3:8.1f} us, best pgemm "
                  f"{best} {med[best] * 1e3:8.1f} us -> {pick}", flush=True)
            if N in GATE_UP:  # the fused gate/up + SiLU GEMM against hipBLASLt + the act kernel
                ya = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
                fc = {"blas+act": lambda: ops.gated_act(F.linear(x, w), ops.ACT_SILU)}
                for v in vs:
                    if v >= 3:
                        fc[(v, False)] = (lambda v=v: ops.pgemm_silu(x, w, variant=v, out=ya))
                fr = {k: [] for k in fc}
                for _ in range(a.rounds):
                    for k, fn in fc.items():
                        fr[k].append(timeit(fn, it))
                fm = {k: sorted(v)[len(v) // 2] for k, v in fr.items()}
                if len(fm) > 1:
                    fb = min((k for k in fm if k != "blas+act"), key=lambda k: fm[k])
                    fp = fb if fm[fb] < (1 - a.margin / 2) * fm["blas+act"] else None
                    rows.append((("silu", mb), N, K, fp, fm[fb] * 1e3, fm["blas+act"] * 1e3))
                    print(f"   fused SiLU: blas+act {fm['blas+act'] * 1e3:8.1f} us, pgemm_silu {fb} "
                          f"{fm[fb] * 1e3:8.1f} us -> {fp}", flush=True)
                del ya
            del x, y
        del w
    with open(a.out, "w") as f:
        f.write('"""Prefill GEMM dispatch table (generated by scripts/make_pgemm_table.py on 1x MI355X,\n'
                f'random operands, {a.rounds} interleaved rounds, margin {a.margin:.0%}).\n\n'
                "(M bucket = ceil(M / 256), N, K) -> ((variant, split_k) or None, best pgemm us, hipBLASLt us).\n"
                "A plan is listed only where the hand-written prefill GEMM (csrc/ops/pgemm.hip) beat\n"
                "hipBLASLt by the margin; None and missing shapes run on hipBLASLt. Static, so every\n"
                'run and every TP / EP rank makes the same choice.\n"""\n\nPGEMM_TABLE = {\n')
        for mb, N, K, pick, ours, blas in rows:
            p = "None" if pick is None else f"({pick[0]}, {pick[1]})"
            key = f"({mb}, {N}, {K})" if isinstance(mb, int) else f"(\"silu\", {mb[1]}, {N}, {K})"
            f.write(f"    {key}: ({p}, {ours:.1f}, {blas:.1f}),\n")
        f.write("}\n")
    print(f"wrote {a.out} ({len(rows)} entries, {sum(1 for r in rows if r[3])} pgemm) in {time.time() - t_start:.0f} s")


if __name__ == "__main__":
    main()
