"""KV-token capacity of one replica at a fixed --gpu-memory-utilization, with and
without the hybrid KV-cache manager (engine/hybrid_kv.py): the full-attention
pool's tokens (what a long prompt can use) and the windowed pool's blocks.
Random-init weights; one engine at a time on one device.

  python scripts/kv_capacity.py [--model gpt-oss-120b] [--quantization fp8] [--util 0.92]
Prints one JSON line.
"""
import argparse
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-oss-120b")
    ap.add_argument("--quantization", default="fp8")
    ap.add_argument("--util", type=float, default=0.92)
    ap.add_argument("--block-size", type=int, default=16)
    a = ap.parse_args()
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine

    out = {"model": a.model, "quantization": a.quantization, "gpu_memory_utilization": a.util}
    for hybrid in (False, True):
        cfg = EngineConfig.create(a.model, device="cuda", block_size=a.block_size, max_num_batched_tokens=8192,
                                  max_num_seqs=256, max_model_len=16384, gpu_memory_utilization=a.util,
                                  quantization=a.quantization, hybrid_kv_cache_manager=hybrid, enforce_eager=True)
        eng = LLMEngine(cfg)
        r = eng.runner
        full_blocks = eng.bm.num_blocks
        rec = {"hybrid": bool(r.hybrid), "full_pool_blocks": int(full_blocks),
               "full_pool_tokens": int(full_blocks * a.block_size),
               "kv_gb": round(r.kv.numel() * r.kv.element_size() / 2**30, 2)}
        if r.hybrid:
            rec["swa_pool_blocks"] = int(r.kv_swa.shape[1])
            rec["swa_gb"] = round(r.kv_swa.numel() * r.kv_swa.element_size() / 2**30, 2)
        out["hybrid" if hybrid else "full_kv"] = rec
        print(json.dumps(rec), flush=True)
        eng.shutdown()
        del eng, r
        gc.collect()
        torch.cuda.empty_cache()
    out["capacity_ratio"] = round(out["hybrid"]["full_pool_tokens"] / out["full_kv"]["full_pool_tokens"], 3)
    print("CAPACITY " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
