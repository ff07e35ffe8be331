"""Shader clock and package power while a prefill GEMM runs back to back (is the
70B prefill GEMM power/clock-limited, or is the matrix pipe idle?).

Each arm loops one GEMM for ~5 s; a side thread samples ``rocm-smi -c -P``
(read-only) every 0.4 s. Printed per arm: achieved TF/s, median sclk, median
power, and TF/s per GHz (the clock-normalised efficiency: the bf16 dense peak
is 2.5 PF/s at 2.4 GHz = 1042 TF/s per GHz).

  python scripts/gemm_clock_probe.py [gemm,attn,moe]
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


def attn_arms():
    """GQA prefill attention (70B heads, one 5000-token causal prompt) and paged decode (B=64, ctx 5000)."""
    import math

    dev = "cuda"
    Hq, Hkv, D, bs, ctx = 64, 8, 128, 64, 5000
    nb = math.ceil(ctx / bs) * 64 + 1
    kc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
    per = math.ceil(ctx / bs)
    bt = torch.randperm(nb - 1, device=dev)[:per].view(1, per).int()
    q = torch.randn(ctx, Hq * D, device=dev, dtype=torch.bfloat16)
    i32 = lambda v: torch.tensor([v], dtype=torch.int32, device=dev)  # noqa: E731
    tpi = ops.prefill_tokens_per_item(Hq, Hkv, D, bs, False)
    items = torch.tensor(ops.build_prefill_items([ctx], [ctx], tpi), dtype=torch.int32, device=dev).view(-1, 2)
    out = torch.empty(ctx, Hq * D, device=dev, dtype=torch.bfloat16)
    fl = 4 * Hq * D * sum(i + 1 for i in range(ctx))
    arm("prefill attention v2 ISL 5000", lambda: ops.paged_prefill(q, kc, vc, bt, i32(0), i32(ctx), i32(ctx), Hq, Hkv,
                                                                    D, D ** -0.5, 0, None, items=items, out=out), fl)
    B = 64
    btd = torch.randperm(nb - 1, device=dev)[:B * per].view(B, per).int()
    qd = torch.randn(B, Hq * D, device=dev, dtype=torch.bfloat16)
    sl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    od = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    split = ops.decode_split_plan(ctx, B, Hkv, Hq // Hkv)
    arm("paged decode B=64 ctx 5000 (flops col = GB/s)",
        lambda: ops.paged_decode(qd, kc, vc, btd, sl, Hq, Hkv, D, D ** -0.5, 0, None, split=split, out=od,
                                 max_ctx=ctx), B * ctx * Hkv * D * 2 * 2 * 1000)


def moe_arms():
    """Block-fp8 and bf16 grouped expert GEMMs (moe4) at DeepSeek EP8 T=4096 and gpt-oss-120b T=5120."""
    dev = "cuda"
    for name, (T, E, k, d, F, act) in {"deepseek-ep8 T=4096": (4096, 32, 8, 7168, 2048, 0),
                                       "gpt-oss-120b T=5120": (5120, 128, 4, 2880, 2880, 2)}.items():
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
        w1 = (torch.randn(E, 2 * F, d, device=dev) * 0.02).to(torch.bfloat16)
        w2 = (torch.randn(E, d, F, device=dev) * 0.02).to(torch.bfloat16)
        w1q, w1s = ops.quant_fp8_block_weight(w1)
        w2q, w2s = ops.quant_fp8_block_weight(w2)
        w1q, w2q = ops.pad_fp8_k(w1q, c128(d)), ops.pad_fp8_k(w2q, c128(F))
        ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
        fl = 2 * T * k * 3 * F * d
        arm(f"MoE fp8 {name}", lambda: ops.moe_experts_fp8(x, ids, wts, w1q, w1s, w2q, w2s, act), fl)
        arm(f"MoE bf16 {name}", lambda: ops.moe_experts(x, ids, wts, w1, w2, act), fl)
        del w1, w2, w1q, w2q
        torch.cuda.empty_cache()


def main():
    dev = "cuda"
    torch.manual_seed(0)
    arms = sys.argv[1].split(",") if len(sys.argv) > 1 else ["gemm"]
    if "attn" in arms:
        attn_arms()
    if "moe" in arms:
        moe_arms()
    if "gemm" not in arms:
        return
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
