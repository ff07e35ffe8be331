"""Multi-LoRA serving: dynamically loaded PEFT adapters served
side by side in one batch.

Every LoRA-able projection (fused qkv, o_proj, fused gate_up, down) holds a
stack of adapter slots A [S, R, in], B [S, out, R] (slot 0 = no adapter,
rank zero-padded to ``--max-lora-rank``, scaling alpha/r folded into B).
Fused projections use one block-diagonal stack: q/k/v (or gate/up) adapters
occupy their own rank ranges of A and the matching row blocks of B, so one
BGMV call serves the fused GEMM. Per step the runner writes each token's slot
into a device vector; the HIP BGMV kernels (csrc/ops/lora.hip) add
B[slot] @ A[slot] @ x row by row - graph-capturable, any mix of adapters.
Under TP, B of column-parallel and A of row-parallel projections are sharded
like the base weights (row-parallel partial sums ride the layer's existing
all-reduce), and load/unload are broadcast to the TP followers.
"""
from __future__ import annotations

import json
import logging
import os
from typing import Optional

import numpy as np
import torch

from llmd_amd import ops
from llmd_amd.parallel.state import get_state

log = logging.getLogger("llmd.lora")


class LoRATarget:
    def __init__(self, mgr: "LoRAManager", S: int, R: int, in_f: int, out_f: int, device):
        self.mgr = mgr
        self.A = torch.zeros(S, R, in_f, dtype=torch.bfloat16, device=device)
        self.B = torch.zeros(S, out_f, R, dtype=torch.bfloat16, device=device)

    def apply(self, y: torch.Tensor, x: torch.Tensor):
        if not self.mgr.active:
            return y
        T = x.shape[0]
        x = x if x.stride(-1) == 1 and x.stride(0) % 8 == 0 else x.contiguous()
        return ops.lora_bgmv(y, x, self.A, self.B, self.mgr.slot_idx[:T])


class LoRAManager:
    def __init__(self, model, max_loras: int, max_rank: int, max_tokens: int, device, broadcast=None):
        self.model = model
        self.S, self.R = max_loras + 1, max_rank
        self.slots: dict[str, int] = {}
        self.paths: dict[str, str] = {}
        self.device = device
        self.slot_idx = torch.zeros(max_tokens, dtype=torch.int32, device=device)
        # kernels always run once LoRA is enabled (slot 0 early-outs), so captured
        # decode graphs stay valid when adapters are loaded later
        self.active = True
        self.broadcast = broadcast   # TP: send load/unload to followers
        st = get_state()
        self.tp, self.rank = st.tp_size, st.tp_rank
        S, R = self.S, self.R
        self.layers = []
        for layer in model.layers:
            a = layer.attn
            t = {"qkv": LoRATarget(self, S, 3 * R, layer.qkv.in_f, layer.qkv.out_f, device),
                 "o": LoRATarget(self, S, R, layer.o_proj.in_f, layer.o_proj.out_f, device)}
            layer.qkv.lora, layer.o_proj.lora = t["qkv"], t["o"]
            mlp = layer.mlp
            if hasattr(mlp, "gate_up"):
                t["gate_up"] = LoRATarget(self, S, 2 * R, mlp.gate_up.in_f, mlp.gate_up.out_f, device)
                t["down"] = LoRATarget(self, S, R, mlp.down.in_f, mlp.down.out_f, device)
                mlp.gate_up.lora, mlp.down.lora = t["gate_up"], t["down"]
            t["geom"] = (a.Hq, a.Hkv, a.D)
            self.layers.append(t)

    # ------------------------------------------------------------ registry
    def names(self) -> list[str]:
        return sorted(self.slots)

    def has(self, name: str) -> bool:
        return name in self.slots

    def id_of(self, name: str) -> int:
        return self.slots[name]

    def name_of(self, slot: int) -> Optional[str]:
        return next((n for n, s in self.slots.items() if s == slot), None)

    # ------------------------------------------------------------ load
    def load(self, name: str, path: Optional[str] = None, slot: Optional[int] = None):
        if name in self.slots:
            raise ValueError(f"LoRA adapter '{name}' is already loaded")
        path = path or name
        if slot is None:
            used = set(self.slots.values())
            free = [s for s in range(1, self.S) if s not in used]
            if not free:
                raise ValueError(f"all {self.S - 1} LoRA slots are in use (--max-loras)")
            slot = free[0]
        if self.broadcast is not None:
            self.broadcast({"lora_cmd": ("load", name, path, slot)})
        self._fill(slot, path)
        self.slots[name], self.paths[name] = slot, path
        log.info("loaded LoRA %s from %s into slot %d", name, path, slot)

    def unload(self, name: str, busy_slots: Optional[set] = None):
        if name not in self.slots:
            raise ValueError(f"LoRA adapter '{name}' is not loaded")
        slot = self.slots[name]
        if busy_slots and slot in busy_slots:
            raise ValueError(f"LoRA adapter '{name}' is in use by running requests")
        if self.broadcast is not None:
            self.broadcast({"lora_cmd": ("unload", name, None, slot)})
        self._clear(slot)
        del self.slots[name], self.paths[name]

    def apply_cmd(self, cmd):
        op, name, path, slot = cmd
        if op == "load":
            self._fill(slot, path)
            self.slots[name], self.paths[name] = slot, path
        else:
            self._clear(slot)
            self.slots.pop(name, None)

    def _clear(self, slot: int):
        for t in self.layers:
            for k, v in t.items():
                if k != "geom":
                    v.A[slot].zero_()
                    v.B[slot].zero_()

    def _fill(self, slot: int, path: str):
        from safetensors import safe_open

        with open(os.path.join(path, "adapter_config.json")) as f:
            acfg = json.load(f)
        r = int(acfg["r"])
        if r > self.R:
            raise ValueError(f"adapter rank {r} > --max-lora-rank {self.R}")
        scale = float(acfg.get("lora_alpha", r)) / r
        self._clear(slot)
        tensors = {}
        with safe_open(os.path.join(path, "adapter_model.safetensors"), framework="pt", device="cpu") as fh:
            for k in fh.keys():
                tensors[k] = fh.get_tensor(k)
        tp, rank = self.tp, self.rank

        def get(i, mod, ab):
            for pre in ("base_model.model.model.layers", "base_model.model.layers", "model.layers"):
                k = f"{pre}.{i}.{mod}.lora_{ab}.weight"
                if k in tensors:
                    return tensors[k].float()
            return None

        def rows(t, n_heads, head_rows):  # this rank's row shard (head granular)
            if n_heads >= tp:
                per = n_heads // tp
                return t[rank * per * head_rows:(rank + 1) * per * head_rows]
            h = rank // (tp // n_heads)
            return t[h * head_rows:(h + 1) * head_rows]

        R = self.R
        for i, t in enumerate(self.layers):
            Hq, Hkv, D = t["geom"]
            Hq_t, Hkv_t = Hq * tp, max(Hkv * tp, 1)
            qkv = t["qkv"]
            off = 0
            for j, (mod, nh) in enumerate((("self_attn.q_proj", Hq_t), ("self_attn.k_proj", Hkv_t),
                                           ("self_attn.v_proj", Hkv_t))):
                A, B = get(i, mod, "A"), get(i, mod, "B")
                nrows = (Hq if j == 0 else Hkv) * D
                if A is not None and B is not None:
                    qkv.A[slot, j * R:j * R + r] = A.to(qkv.A.dtype).to(qkv.A.device)
                    qkv.B[slot, off:off + nrows, j * R:j * R + r] = (rows(B, nh, D) * scale).to(
                        qkv.B.dtype).to(qkv.B.device)
                off += nrows
            A, B = get(i, "self_attn.o_proj", "A"), get(i, "self_attn.o_proj", "B")
            if A is not None and B is not None:
                t["o"].A[slot, :r] = A.chunk(tp, 1)[rank].to(t["o"].A.dtype).to(self.device)
                t["o"].B[slot, :, :r] = (B * scale).to(t["o"].B.dtype).to(self.device)
            if "gate_up" in t:
                gu = t["gate_up"]
                F_local = gu.B.shape[1] // 2
                for j, mod in enumerate(("mlp.gate_proj", "mlp.up_proj")):
                    A, B = get(i, mod, "A"), get(i, mod, "B")
                    if A is not None and B is not None:
                        gu.A[slot, j * R:j * R + r] = A.to(gu.A.dtype).to(self.device)
                        gu.B[slot, j * F_local:(j + 1) * F_local, j * R:j * R + r] = (
                            B.chunk(tp, 0)[rank] * scale).to(gu.B.dtype).to(self.device)
                A, B = get(i, "mlp.down_proj", "A"), get(i, "mlp.down_proj", "B")
                if A is not None and B is not None:
                    t["down"].A[slot, :r] = A.chunk(tp, 1)[rank].to(t["down"].A.dtype).to(self.device)
                    t["down"].B[slot, :, :r] = (B * scale).to(t["down"].B.dtype).to(self.device)

    # ------------------------------------------------------------ per step
    def set_tokens(self, lora_ids, offset: int = 0):
        ids = np.asarray(lora_ids, dtype=np.int32)
        n = len(ids)
        if n:
            src = torch.from_numpy(ids)
            if self.slot_idx.is_cuda:
                src = src.pin_memory()
            self.slot_idx[offset:offset + n].copy_(src, non_blocking=True)


def save_peft_adapter(path: str, tensors: dict, r: int, alpha: float, targets: list[str]):
    """Write a PEFT-format adapter (tests/tools)."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "adapter_config.json"), "w") as f:
        json.dump({"r": r, "lora_alpha": alpha, "target_modules": targets, "peft_type": "LORA"}, f)
    save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(path, "adapter_model.safetensors"))
