"""Per-step attention metadata for a mixed (decode + chunked-prefill) batch.

Token layout of a step: all decode tokens first (one per decoding sequence),
then the prefill chunks back to back. The decode part can be replayed from a
captured hipGraph (static buffers, fixed split plan); the prefill part is
always eager.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class AttnMeta:
    num_tokens: int
    positions: torch.Tensor          # [T] int64
    slot_mapping: torch.Tensor       # [T] int64 (-1 = do not write)
    # decode part
    num_decode: int = 0
    d_block_tables: Optional[torch.Tensor] = None  # [Bd, W] int32
    d_seq_lens: Optional[torch.Tensor] = None      # [Bd] int32
    d_split: Optional[tuple] = None                # (split_size, nsplit)
    d_workspace: Optional[tuple] = None            # (part_o, part_ml)
    d_max_ctx: int = 0
    d_cascade: Optional[tuple] = None              # shared-prefix decode (ops.cascade_tensors)
    d_split_dev: Optional[torch.Tensor] = None     # [1] int32 keys per split, set per graph replay
    # prefill part
    num_prefill_tokens: int = 0
    p_block_tables: Optional[torch.Tensor] = None  # [Bp, W] int32
    p_q_start: Optional[torch.Tensor] = None       # [Bp] int32 (relative to the prefill part)
    p_q_len: Optional[torch.Tensor] = None
    p_ctx_len: Optional[torch.Tensor] = None
    p_items: Optional[torch.Tensor] = None         # [n, 2] int32
    p_items_per_window: Optional[dict] = None
    # MLA (one attention row per decode sequence / prefill token)
    mla_d_rows: Optional[torch.Tensor] = None      # [Bd] int32 = arange (row -> d_block_tables row)
    mla_split: Optional[tuple] = None              # fixed (split_size, nsplit) under graph capture
    mla_workspace: Optional[tuple] = None
    mla_split_dev: Optional[torch.Tensor] = None   # [1] int32 keys per split, set per graph replay
    p_row_seq: Optional[torch.Tensor] = None       # [Tp] int32 prefill token -> p_block_tables row
    p_row_len: Optional[torch.Tensor] = None       # [Tp] int32 keys visible (= position + 1)
    p_max_ctx: int = 0
    # multimodal: step rows that are image placeholders and their embeddings
    mm_rows: Optional[torch.Tensor] = None         # [n] int64
    mm_embeds: Optional[torch.Tensor] = None       # [n, d_model]
    # hybrid KV cache (engine/hybrid_kv.py): the windowed layers' own slot mapping and
    # block tables (everything else shared), or None
    swa: Optional["AttnMeta"] = None

    @property
    def has_prefill(self) -> bool:
        return self.num_prefill_tokens > 0
