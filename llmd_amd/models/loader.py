"""Checkpoint loading: HuggingFace safetensors -> TP-sharded
modules, and the inverse export (TP=1) used by tests and tools.

Each model class describes its parameters with ``weight_specs()``: a list of
``(hf_name, param, kind, extra)`` entries where ``kind`` says how a full
checkpoint tensor maps onto this rank's shard:

  replicate            copy as is (norms, q/k norms, router)
  col                  split dim 0 into tp chunks (column-parallel weight/bias)
  row                  split dim 1 into tp chunks (row-parallel weight)
  vocab                rows [rank*per, rank*per+per) of a vocab-parallel table
                       (zero-padded past the vocabulary)
  rows                 rows start::step of the param (gate/up interleaving of MoE w1)
  experts(_t)          rows [lo, lo+n) of a stacked [E, ...] expert tensor (optionally
                       transposed per expert: HF gpt-oss stores [E, in, out])
  fused                a slice [off, off+len) of a fused column-parallel param
                       (q|k|v or gate|up); ``extra = (off, n_heads_total,
                       head_rows)`` - heads are split across ranks, KV heads
                       replicated when there are fewer KV heads than ranks.

Expert weights may also come as MXFP4 ``<name>_blocks`` / ``<name>_scales`` pairs (the format the
gpt-oss checkpoints ship their experts in): they are dequantised per expert on load.

Only safetensors are read (``safe_open``: no pickle, nothing executed).
"""
from __future__ import annotations

import glob
import os

import torch

from llmd_amd.parallel.state import get_state


def _files(path: str) -> list[str]:
    if os.path.isdir(path):
        fs = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not fs:
            raise FileNotFoundError(f"no *.safetensors under {path}")
        return fs
    return [path]


def _shard_heads(t: torch.Tensor, n_heads: int, head_rows: int, tp: int, rank: int) -> torch.Tensor:
    """Rows of this rank's heads from a [n_heads*head_rows, ...] tensor."""
    if n_heads >= tp:
        per = n_heads // tp
        return t[rank * per * head_rows:(rank + 1) * per * head_rows]
    h = rank // (tp // n_heads)  # fewer heads than ranks: replicate
    return t[h * head_rows:(h + 1) * head_rows]


def place(param: torch.Tensor, full: torch.Tensor, kind: str, extra=None):
    st = get_state()
    tp, rank = st.tp_size, st.tp_rank
    full = full.to(param.dtype)
    with torch.no_grad():
        if kind == "replicate":
            param.copy_(full.view_as(param))
        elif kind == "col":
            param.copy_(full.chunk(tp, 0)[rank])
        elif kind == "row":
            param.copy_(full.chunk(tp, 1)[rank])
        elif kind == "vocab":
            per = param.shape[0]
            part = full[rank * per:(rank + 1) * per]
            param.zero_()
            param[: part.shape[0]].copy_(part)
        elif kind == "fused":
            off, n_heads, head_rows = extra
            part = _shard_heads(full, n_heads, head_rows, tp, rank)
            param[off:off + part.shape[0]].copy_(part)
        elif kind in ("experts", "experts_t"):  # [E, ...] stacked experts -> this rank's slice
            if isinstance(extra, list):  # explicit logical experts per physical slot (EPLB replicas)
                part = full[extra]
            else:
                lo, n = extra
                part = full[lo:lo + n]
            param.copy_(part.transpose(1, 2) if kind == "experts_t" else part)
        elif kind == "rows":  # interleaved rows (gate/up pairs of a fused expert weight)
            start, step = extra
            param[start::step].copy_(full)
        else:
            raise ValueError(kind)


def _mxfp4_experts(param: torch.Tensor, blocks: torch.Tensor, scales: torch.Tensor, extra) -> None:
    """MXFP4 expert tensors as gpt-oss checkpoints ship them: ``<name>_blocks`` uint8 [E, out, K/32, 16]
    (32 e2m1 codes per block, element 2i in the low nibble) and ``<name>_scales`` uint8 [E, out, K/32]
    (E8M0, bias 127) -> this rank's experts dequantised into ``param`` [E_local, out, K] one expert at a
    time on the param's device. ``--quantization mxfp4`` re-quantises them afterwards without loss: every
    element gets its checkpoint value back (a block's scale may come back one step lower with doubled
    codes; models/layers.py quantize_mxfp4, tests/test_moe_mxfp4.py)."""
    from llmd_amd import ops

    sel = extra if isinstance(extra, list) else list(range(extra[0], extra[0] + extra[1]))
    E, N, nb, w = blocks.shape
    if w != 16 or scales.shape != (E, N, nb) or param.shape[0] != len(sel) or tuple(param.shape[1:]) != (N, nb * 32):
        raise ValueError(f"MXFP4 tensor shapes {tuple(blocks.shape)} / {tuple(scales.shape)} do not fit "
                         f"the parameter {tuple(param.shape)}")
    with torch.no_grad():
        for i, e in enumerate(sel):
            q = blocks[e].reshape(1, N, nb * 16).to(param.device)
            param[i].copy_(ops.dequant_mxfp4_weight(q, scales[e:e + 1].to(param.device))[0])


def load_weights(model: torch.nn.Module, path: str, strict: bool = True) -> int:
    from contextlib import ExitStack

    from safetensors import safe_open

    specs = {name: (p, kind, extra) for name, p, kind, extra in model.weight_specs()}
    seen = set()
    with ExitStack() as stack:
        where = {}
        for f in _files(path):
            fh = stack.enter_context(safe_open(f, framework="pt", device="cpu"))
            for name in fh.keys():
                where[name] = fh
        for name, fh in where.items():
            key = name if name in specs else "model." + name  # base-model checkpoints (e.g. facebook/opt-*)
            if key not in specs:
                continue
            p, kind, extra = specs[key]
            place(p, fh.get_tensor(name).to(p.device), kind, extra)
            seen.add(key)
        for key, (p, kind, extra) in specs.items():  # experts stored as MXFP4 blocks + scales
            if key in seen or kind not in ("experts", "experts_t"):
                continue
            for base in (key, key[6:] if key.startswith("model.") else None):
                if base and base + "_blocks" in where and base + "_scales" in where:
                    _mxfp4_experts(p, where[base + "_blocks"].get_tensor(base + "_blocks"),
                                   where[base + "_scales"].get_tensor(base + "_scales"), extra)
                    seen.add(key)
                    break
    missing = set(specs) - seen
    if missing and strict:
        raise KeyError(f"checkpoint is missing {len(missing)} tensors, e.g. {sorted(missing)[:4]}")
    return len(seen)


def export_hf(model: torch.nn.Module) -> dict[str, torch.Tensor]:
    """Full HF-named state dict of a TP=1 model (inverse of load_weights)."""
    if get_state().tp_size != 1:
        raise RuntimeError("export_hf needs tp_size == 1")
    out: dict[str, torch.Tensor] = {}
    for name, p, kind, extra in model.weight_specs():
        if kind == "fused":
            off, n_heads, head_rows = extra
            out[name] = p[off:off + n_heads * head_rows].detach().cpu().clone()
        elif kind == "vocab":
            out[name] = p[: model.cfg.vocab_size].detach().cpu().clone()
        elif kind == "rows":
            start, step = extra
            out[name] = p[start::step].detach().cpu().clone()
        elif kind == "experts_t":
            out[name] = p.transpose(1, 2).detach().cpu().contiguous()
        else:
            out[name] = p.detach().cpu().clone()
    return out


def save_safetensors(tensors: dict[str, torch.Tensor], path: str):
    from safetensors.torch import save_file

    save_file({k: v.contiguous() for k, v in tensors.items()}, path)
