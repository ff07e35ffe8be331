"""Request, sampling parameters and per-step outputs."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Any, Optional


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    min_tokens: int = 0
    seed: Optional[int] = None
    stop_token_ids: list[int] = field(default_factory=list)
    stop: list[str] = field(default_factory=list)
    ignore_eos: bool = False
    logprobs: Optional[int] = None
    n: int = 1
    embed: bool = False  # /v1/embeddings: keep the final hidden state of the last prompt token
    presence_penalty: float = 0.0      # OpenAI: - p for every token already generated
    frequency_penalty: float = 0.0     # OpenAI: - f x count of the token in the output
    repetition_penalty: float = 1.0    # vLLM/HF: logits of prompt+output tokens / r (if > 0) or x r
    min_p: float = 0.0                 # drop tokens with prob < min_p x max prob
    logit_bias: Optional[dict] = None  # token id -> additive bias

    @property
    def penalized(self) -> bool:
        return bool(self.presence_penalty or self.frequency_penalty or self.repetition_penalty != 1.0
                    or self.logit_bias or self.min_p > 0.0)

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0

    @classmethod
    def from_openai(cls, body: dict, default_max: int = 16, vocab_size: Optional[int] = None) -> "SamplingParams":
        stop = body.get("stop") or []
        if isinstance(stop, str):
            stop = [stop]
        mt = body.get("max_completion_tokens", body.get("max_tokens"))

        def g(k, d):
            v = body.get(k)
            return d if v is None else v
        sp = cls(
            max_tokens=int(mt) if mt is not None else default_max,
            temperature=float(body.get("temperature", 1.0) if body.get("temperature") is not None else 1.0),
            top_p=float(g("top_p", 1.0)),
            top_k=int(body.get("top_k", 0) or 0),
            min_tokens=int(body.get("min_tokens", 0) or 0),
            seed=body.get("seed"),
            stop_token_ids=list(body.get("stop_token_ids") or []),
            stop=stop,
            ignore_eos=bool(body.get("ignore_eos", False)),
            logprobs=body.get("logprobs") if isinstance(body.get("logprobs"), int) else (
                1 if body.get("logprobs") is True else None),
            n=int(g("n", 1)),
            presence_penalty=float(g("presence_penalty", 0.0)),
            frequency_penalty=float(g("frequency_penalty", 0.0)),
            repetition_penalty=float(g("repetition_penalty", 1.0)),
            min_p=float(g("min_p", 0.0)),
            logit_bias={int(k): float(v) for k, v in (body.get("logit_bias") or {}).items()} or None,
        )._validated()
        return sp.check_vocab(vocab_size) if vocab_size else sp

    def _validated(self) -> "SamplingParams":
        """OpenAI / vLLM ranges (ValueError -> HTTP 400)."""
        if not -2.0 <= self.presence_penalty <= 2.0:
            raise ValueError(f"presence_penalty must be in [-2, 2], got {self.presence_penalty}")
        if not -2.0 <= self.frequency_penalty <= 2.0:
            raise ValueError(f"frequency_penalty must be in [-2, 2], got {self.frequency_penalty}")
        if self.repetition_penalty <= 0.0:
            raise ValueError(f"repetition_penalty must be > 0, got {self.repetition_penalty}")
        if not 0.0 <= self.min_p <= 1.0:
            raise ValueError(f"min_p must be in [0, 1], got {self.min_p}")
        if not 1 <= self.n <= 128:
            raise ValueError(f"n must be in [1, 128], got {self.n}")
        if self.max_tokens < 0 or self.temperature < 0 or not 0.0 < self.top_p <= 1.0:
            raise ValueError("max_tokens and temperature must be >= 0 and top_p in (0, 1]")
        for k, v in (self.logit_bias or {}).items():
            if k < 0:
                raise ValueError(f"logit_bias token id {k} is negative")
            if not -100.0 <= v <= 100.0:  # OpenAI range; also rejects nan/inf
                raise ValueError(f"logit_bias value for token {k} must be in [-100, 100], got {v}")
        return self

    def check_vocab(self, vocab_size: int) -> "SamplingParams":
        """logit_bias keys index the logits row on the GPU and must lie in
        [0, vocab_size): an out-of-range column in the penalty index_put_ would
        fault the device for every in-flight request."""
        for k in (self.logit_bias or {}):
            if not 0 <= k < vocab_size:
                raise ValueError(f"logit_bias token id {k} outside the vocabulary [0, {vocab_size})")
        return self


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    PREEMPTED = 2
    WAITING_FOR_REMOTE_KV = 3
    FINISHED_STOPPED = 10
    FINISHED_LENGTH = 11
    FINISHED_ABORTED = 12
    FINISHED_ERROR = 13

    @property
    def finished(self) -> bool:
        return self.value >= 10


FINISH_REASON = {
    Status.FINISHED_STOPPED: "stop",
    Status.FINISHED_LENGTH: "length",
    Status.FINISHED_ABORTED: "abort",
    Status.FINISHED_ERROR: "error",
}

_seq_counter = itertools.count(1)


@dataclass
class Request:
    request_id: str
    prompt_token_ids: list[int]
    params: SamplingParams = field(default_factory=SamplingParams)
    priority: int = 0
    arrival_time: float = field(default_factory=time.monotonic)
    lora_id: int = 0
    # P/D disaggregation (vLLM NixlConnector-compatible kv_transfer_params)
    kv_transfer_params: Optional[dict] = None
    status: Status = Status.WAITING
    output_token_ids: list[int] = field(default_factory=list)
    output_logprobs: list[float] = field(default_factory=list)
    num_computed_tokens: int = 0
    num_cached_tokens: int = 0
    num_preemptions: int = 0
    seq_id: int = field(default_factory=lambda: next(_seq_counter))
    # timing (monotonic seconds)
    first_scheduled_time: Optional[float] = None
    first_token_time: Optional[float] = None
    last_token_time: Optional[float] = None
    finished_time: Optional[float] = None
    stop_reason: Any = None
    extra: dict = field(default_factory=dict)
    # multimodal inputs (models/vision.py MMInput): image placeholder runs + embeddings
    mm_inputs: Optional[list] = None
    # async scheduling (engine.py): the last output token is a placeholder whose value is
    # still on the device (its step is in flight); final_pending = that token is the last one
    # (max_tokens / max_model_len reached), so the request is not scheduled again
    async_pending: bool = False
    final_pending: bool = False

    @property
    def cache_extra(self) -> int:
        """Block-key namespace: LoRA adapter and, for multimodal prompts, the images."""
        if not self.mm_inputs:
            return self.lora_id
        from llmd_amd.models.vision import mm_cache_key

        return (mm_cache_key(self.mm_inputs) ^ (self.lora_id * 0x9E3779B97F4A7C15)) & ((1 << 63) - 1)

    @property
    def all_token_ids(self) -> list[int]:
        return self.prompt_token_ids + self.output_token_ids

    def token_at(self, i: int) -> int:
        """Token i of prompt+output without materialising the concatenation
        (the per-step decode path must stay O(1) in the context length)."""
        n = len(self.prompt_token_ids)
        return self.prompt_token_ids[i] if i < n else self.output_token_ids[i - n]

    def token_range(self, a: int, b: int) -> list[int]:
        n = len(self.prompt_token_ids)
        if b <= n:
            return self.prompt_token_ids[a:b]
        if a >= n:
            return self.output_token_ids[a - n:b - n]
        return self.prompt_token_ids[a:] + self.output_token_ids[:b - n]

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_token_ids) + len(self.output_token_ids)

    @property
    def num_prompt_tokens(self) -> int:
        return len(self.prompt_token_ids)

    @property
    def is_prefill(self) -> bool:
        return self.num_computed_tokens < self.num_tokens - 1 or not self.output_token_ids and \
            self.num_computed_tokens < self.num_prompt_tokens

    @property
    def finish_reason(self) -> Optional[str]:
        return FINISH_REASON.get(self.status)


@dataclass
class RequestOutput:
    request_id: str
    new_token_ids: list[int]
    new_logprobs: list[float]
    finished: bool
    finish_reason: Optional[str]
    num_prompt_tokens: int
    num_output_tokens: int
    num_cached_tokens: int = 0
    kv_transfer_params: Optional[dict] = None
    embedding: Optional[list] = None
    ttft: Optional[float] = None
    metrics: Optional[dict] = None
