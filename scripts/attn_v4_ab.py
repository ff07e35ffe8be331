"""A/B of the prefill attention kernels v2 (16x16x32) and v4 (32x32x16) at the serving shapes
(Llama-3-70B heads 64/8, D 128, block 64): ISL 5000 and 8192 fresh prompts and a 4096 chunk over
a 4096 prefix, interleaved rounds in one process (LLMD_PREFILL_V4 is read per launch).
  python scripts/attn_v4_ab.py [--rounds 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_attn import prefill  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    cases = [(5000, 5000), (8192, 8192), (8192, 4096), (2048, 2048)]
    res = {}
    arms = {"v2": ("0", "3"), "v4-builtin-dma": ("1", "1"), "v4-asm-dma": ("1", "3"), "v4-pipelined": ("1", "7")}
    for r in range(a.rounds):
        for ctx, ql in cases:
            for name, (on, var) in arms.items():
                os.environ["LLMD_PREFILL_V4"] = on
                os.environ["LLMD_PREFILL_V4_VARIANT"] = var
                t = prefill(ctx, ql, 64, 8, 128, 64, check=(r == 0 and ctx == 2048))
                res.setdefault((ctx, ql, name), []).append(t)
    for ctx, ql in cases:
        vis = sum(ctx - ql + i + 1 for i in range(ql))
        fl = 4 * 64 * 128 * vis
        med = {n: sorted(res[(ctx, ql, n)])[a.rounds // 2] for n in arms}
        print(f"AB ctx={ctx} q={ql}: " + " | ".join(f"{n} {t * 1e3:.3f} ms {fl / t / 1e12:.0f} TF/s"
                                                   for n, t in med.items()), flush=True)


if __name__ == "__main__":
    main()
