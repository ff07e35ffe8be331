"""Prefill attention kernel only (ISL 5000, Llama-3-70B heads), for counter collection."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_attn import prefill  # noqa: E402

if __name__ == "__main__":
    for _ in range(2):
        prefill(5000, 5000, 64, 8, 128, 64)
    torch.cuda.synchronize()
