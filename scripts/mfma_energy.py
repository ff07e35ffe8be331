"""Energy per FLOP of bf16 MFMA shapes at the package power cap (scripts/probes/mfma_energy.hip):
register-only MFMA streams, one launch looped ~5 s per arm while rocm-smi samples clock + power.
Both shapes do 262144 FLOPs per wave per iteration (16 x 16x16x32 or 8 x 32x32x16).
  python scripts/mfma_energy.py"""
import ctypes
import os
import statistics
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_clock_probe import sample  # noqa: E402

LIB = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probes", "mfma_energy.so"))


def arm(name, shape, zero, iters=20000, blocks=1024, secs=5.0):
    out = torch.empty(blocks * 256, device="cuda")
    fl = blocks * 4 * 262144 * iters  # 4 waves per block, 262144 FLOPs per wave per iteration in both shapes
    go = lambda: LIB.mfma_burn_launch(ctypes.c_void_p(out.data_ptr()), shape, zero, iters, blocks)  # noqa: E731
    assert go() == 0
    torch.cuda.synchronize()
    samples, stop = [], threading.Event()
    th = threading.Thread(target=sample, args=(stop, samples))
    n, t0 = 0, time.perf_counter()
    th.start()
    while time.perf_counter() - t0 < secs:
        go()
        n += 1
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stop.set()
    th.join()
    tf = fl * n / dt / 1e12
    sk = statistics.median(s for s, _ in samples)
    pw = statistics.median(p for _, p in samples)
    print(f"{name:34s} {tf:7.0f} TF/s  sclk {sk:6.0f} MHz  power {pw:6.0f} W  {tf / (sk / 1000):6.0f} TF/s per GHz  "
          f"{pw / tf:.3f} pJ/FLOP ({len(samples)} samples)", flush=True)


if __name__ == "__main__":
    arm("16x16x32 bf16 random", 0, 0)
    arm("32x32x16 bf16 random", 1, 0)
    arm("16x16x32 bf16 zero", 0, 1)
    arm("32x32x16 bf16 zero", 1, 1)
    arm("16x16x32 bf16 random (again)", 0, 0)
