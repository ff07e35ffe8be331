"""Pre-tuned dense GEMM selection (the reference ships tuned
GEMM configs per GPU for its serving images; here the plain projections run
through hipBLASLt and PyTorch TunableOp picks the solution per shape).

`scripts/tune_gemm.py` searches hipBLASLt/rocBLAS solutions for the serving
shapes on an MI355X and writes a TunableOp CSV; `llmd_amd/tuning/` keeps the
committed results. `enable_lookup()` turns TunableOp on in lookup-only mode
(tuning disabled, so nothing new is written at exit), so a served step or a hipGraph
capture never triggers a search; shapes absent from the file keep
hipBLASLt's default heuristic.
"""
from __future__ import annotations

import os

import torch

TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")
_enabled: str | None = None


def model_gemm_shapes(model: str, tp: int = 1) -> dict:
    """(N, K) of the dense projections of a preset model at tensor-parallel size tp."""
    from ..engine.config import get_model_config

    c = get_model_config(model)
    D = c.head_dim or c.hidden_size // c.num_attention_heads
    d, F = c.hidden_size, c.intermediate_size
    q, kv = c.num_attention_heads * D // tp, max(1, c.num_key_value_heads // tp) * D
    return {"qkv": (q + 2 * kv, d), "o": (d, q), "gate_up": (2 * F // tp, d), "down": (d, F // tp),
            "lm_head": (c.vocab_size // tp, d)}


def tuning_file(arch: str | None = None) -> str:
    if arch is None:
        arch = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    return os.path.join(TUNING_DIR, f"tunableop_{arch}.csv")


def enable_lookup(path: str | None = None) -> str | None:
    """Enable TunableOp lookup from the committed results for this GPU arch.
    Returns the file used, or None (no GPU, opt-out LLMD_GEMM_TUNING=0, or no file)."""
    global _enabled
    if os.environ.get("LLMD_GEMM_TUNING", "1") == "0" or not torch.cuda.is_available():
        return None
    if _enabled is not None:
        return _enabled
    path = path or tuning_file()
    if not os.path.exists(path):
        return None
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    tun.set_filename(path)
    tun.read_file(path)
    _enabled = path
    return path
