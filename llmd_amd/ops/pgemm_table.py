"""Prefill GEMM dispatch table (placeholder until scripts/make_pgemm_table.py has
run on the GPU): empty, so every prefill GEMM runs on hipBLASLt.

(M bucket = ceil(M / 256), N, K) -> ((variant, split_k) or None, best pgemm us, hipBLASLt us).
"""

PGEMM_TABLE = {}
