"""Tokenizers: HF ``tokenizers`` from a local directory, or a byte-level
fallback (no network: synthetic/random-weight deployments use the fallback).

Also provides the chat template rendering used by ``/v1/chat/completions``
and ``/v1/chat/completions/render`` (the render endpoint the router's
token-producer calls).
"""
from __future__ import annotations

import json
import os
from typing import Optional


class ByteTokenizer:
    """UTF-8 bytes -> ids [offset, offset+256); special ids below offset."""

    def __init__(self, vocab_size: int, bos_id: int = 1, eos_id: int = 2, offset: int = 3):
        self.vocab_size = vocab_size
        self.bos_token_id = bos_id
        self.eos_token_id = eos_id
        self.offset = offset if vocab_size > 259 else 0

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = [b + self.offset for b in text.encode("utf-8")]
        return ([self.bos_token_id] if add_bos else []) + ids

    def decode(self, ids, skip_special: bool = True) -> str:
        bs = bytes((i - self.offset) & 0xFF for i in ids
                   if self.offset <= i < self.offset + 256 or not skip_special)
        return bs.decode("utf-8", errors="replace")


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        f = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
        self.tok = Tokenizer.from_file(f)
        self.vocab_size = self.tok.get_vocab_size()
        cfgp = os.path.join(os.path.dirname(f), "tokenizer_config.json")
        self.bos_token_id = self.eos_token_id = None
        self.chat_template = None
        if os.path.exists(cfgp):
            with open(cfgp) as fh:
                c = json.load(fh)
            for k in ("bos_token", "eos_token"):
                v = c.get(k)
                if isinstance(v, dict):
                    v = v.get("content")
                if v is not None:
                    setattr(self, k + "_id", self.tok.token_to_id(v))
            self.chat_template = c.get("chat_template")

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        if add_bos and self.bos_token_id is not None:
            ids = [self.bos_token_id] + ids
        return ids

    def decode(self, ids, skip_special: bool = True) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=skip_special)


def load_tokenizer(path: Optional[str], vocab_size: int, bos: int = 1, eos: int = 2):
    if path and os.path.exists(path):
        try:
            return HFTokenizer(path)
        except Exception:  # pragma: no cover - corrupt tokenizer file
            pass
    return ByteTokenizer(vocab_size, bos_id=bos if bos < 3 else 1, eos_id=eos if eos < 3 else 2)


def render_chat(messages: list[dict], add_generation_prompt: bool = True, style: str = "llama3",
                tools=None) -> str:
    """Built-in chat template of one model family (``serving/chat_template.py``)."""
    from .chat_template import BUILTIN

    return BUILTIN[style](messages, add_generation_prompt, tools)
