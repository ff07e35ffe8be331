"""Steady-state windows for the closed-loop serving benchmarks (bench.py,
bench_pd.py).

In a closed loop with R requests in flight and OSL output tokens each, every
engine step emits (about) R tokens, so R/OSL requests complete per step and
as many replacement prompts must be prefilled per step: conservation. A timed
window of K steps is steady state only if it holds K*R/OSL prefills.

The setup phase cannot give that by itself: requests are admitted over a
ramp (one prompt-sized chunk per step), so their remaining output lengths are
bunched and the first completions arrive late (the 70B driver
window had 4 prefill steps in 20 where conservation requires 5.1, which
overstated throughput by ~20 %). ``restagger`` fixes the phase at the end of
setup: the running requests, oldest first, get ``ceil((i+1)*OSL/R)`` output
tokens left, so completion i lands on step ceil((i+1)*OSL/R) and the
completions (hence the replacement prefills) arrive at exactly R/OSL per step
from the first step after setup on. A replacement runs OSL steps (one prefill
step + OSL-1 decode steps), so the pattern repeats with period OSL.

The reference benchmarks its P/D path at a steady request rate for the same
reason (guides/pd-disaggregation/README.md:331-470: 5400 requests over 120 s).
"""
from __future__ import annotations

import math


def remaining_schedule(n: int, osl: int, concurrency: int) -> list[int]:
    """Output tokens left for the n oldest in-flight requests (oldest first)."""
    return [max(1, math.ceil((i + 1) * osl / concurrency)) for i in range(n)]


def restagger(running, osl: int, concurrency: int) -> int:
    """Re-set ``params.max_tokens`` of the running requests (those past their
    prefill) so their completions are evenly spaced, R/OSL per step. Oldest
    (most tokens generated) first. Returns the largest total output length
    assigned (the caller's max_model_len must allow prompt + that)."""
    reqs = sorted((r for r in running if r.output_token_ids), key=lambda r: (-len(r.output_token_ids), r.seq_id))
    longest = 0
    for r, left in zip(reqs, remaining_schedule(len(reqs), osl, concurrency)):
        r.params.max_tokens = len(r.output_token_ids) + left
        # async scheduling: a request whose in-flight token was its last under the old length
        # is scheduled again under the new one
        r.final_pending = len(r.output_token_ids) >= r.params.max_tokens
        longest = max(longest, r.params.max_tokens)
    return longest


def expected_prefills(steps: int, concurrency: int, osl: int) -> float:
    """Prefills a steady-state window of ``steps`` steps must hold."""
    return steps * concurrency / osl


def window_report(prefills: int, steps: int, concurrency: int, osl: int) -> dict:
    exp = expected_prefills(steps, concurrency, osl)
    return {"prefills_in_window": int(prefills), "conservation_prefills": round(exp, 2),
            "within_one": abs(prefills - exp) <= 1.0}
