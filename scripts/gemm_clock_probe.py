"""Shader clock and package power while a prefill GEMM runs back to back (is the
70B prefill GEMM power/clock-limited, or is the matrix pipe idle?).

Each arm loops one GEMM for ~5 s; a side thread samples ``rocm-smi -c -P``
(read-only) every 0.4 s. Printed per arm: achieved TF/s, median sclk, median
power, and TF/s per GHz (the clock-normalised efficiency: the bf16 dense peak
is 2.5 PF/s at 2.4 GHz = 1042 TF/s per GHz).

  python scripts/gemm_clock_probe.py
"""
import os
import re
import statistics
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd import ops  # noqa: E402


def sample(stop, out):
    while not stop.is_set():
        try:
            txt = subprocess.run(["rocm-smi", "-c", "-P"], capture_output=True, text=True, timeout=5).stdout
        except (OSError, subprocess.TimeoutExpired):
            txt = ""
        if not out and not getattr(sample, "shown", False):
            sample.shown = True
            print(txt, flush=True)
        s = re.search(r"sclk clock level:.*?\((\d+)\s*Mhz\)", txt, re.I)
        p = re.search(r"Power \(W\):\s*([\d.]+)", txt)
        if s:
            out.append((float(s.group(1)), float(p.group(1)) if p else float("nan")))
        time.sleep(0.4)


def arm(name, fn, flops, secs=5.0):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    samples = []
    stop = threading.Event()
    th = threading.Thread(target=sample, args=(stop, samples))
    n = 0
    t0 = time.perf_counter()
    th.start()
    while time.perf_counter() - t0 < secs:
        for _ in range(10):
            fn()
        n += 10
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stop.set()
    th.join()
    tf = flops * n / dt / 1e12
    sk = statistics.median(s for s, _ in samples) if samples else float("nan")
    pw = statistics.median(p for _, p in samples) if samples else float("nan")
    print(f"{name:40s} {dt / n * 1e6:9.1f} us  {tf:7.0f} TF/s  sclk {sk:6.0f} MHz  power {pw:6.0f} W  "
          f"{tf / (sk / 1000):6.0f} TF/s per GHz  ({len(samples)} samples)", flush=True)


def main():
    dev = "cuda"
    torch.manual_seed(0)
    K = 8192
    for M in (5063, 4608):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        wgu = torch.randn(57344, K, device=dev, dtype=torch.bfloat16) * 0.02
        y = torch.empty(M, 28672, device=dev, dtype=torch.bfloat16)
        fl = 2 * M * 57344 * K
        arm(f"M={M} gate_up pgemm_silu (v3)", lambda: ops.pgemm_silu(x, wgu, variant=3, out=y), fl)
        arm(f"M={M} gate_up hipBLASLt", lambda: torch.mm(x, wgu.t()), fl)
        del wgu, y
        xd = torch.randn(M, 28672, device=dev, dtype=torch.bfloat16)
        wd = torch.randn(K, 28672, device=dev, dtype=torch.bfloat16) * 0.02
        yd = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        fl = 2 * M * K * 28672
        arm(f"M={M} down pgemm (v3 split)", lambda: ops.pgemm(xd, wd, out=yd, variant=3, split_k=True), fl)
        arm(f"M={M} down hipBLASLt", lambda: torch.mm(xd, wd.t()), fl)
        del xd, wd, yd
        torch.cuda.empty_cache()
    # zeros: the same GEMM with no bit toggling (power floor of the data path)
    M = 5063
    x = torch.zeros(M, K, device=dev, dtype=torch.bfloat16)
    wgu = torch.zeros(57344, K, device=dev, dtype=torch.bfloat16)
    y = torch.empty(M, 28672, device=dev, dtype=torch.bfloat16)
    arm(f"M={M} gate_up pgemm_silu ZERO operands", lambda: ops.pgemm_silu(x, wgu, variant=3, out=y),
        2 * M * 57344 * K)


if __name__ == "__main__":
    main()
