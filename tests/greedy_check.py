"""Greedy-output comparison for parallel-layout tests (TP / EP / DBO against a
single-process engine on the same weights).

Tiny random-init models have near-flat logits, and a parallel layout sums in
another order (TP all-reduce, EP combine, micro-batch halves) in bf16, so a
greedy argmax can flip between two almost-equal logits - and from there the
contexts differ. A sequence passes when it matches the reference, or when its
FIRST divergence is a near-tie of the reference: the reference's logit for its
own token exceeds the logit of ours by at most max(abs_tol, rel_tol * max|logit|)
(probed by re-running the reference on the common prefix). Later tokens are
not compared. A real layout bug (wrong shard, wrong expert, dropped rows)
diverges with large margins and fails.
"""
from __future__ import annotations

from llmd_amd.engine.request import SamplingParams


def first_divergences(ref, prompts, got, want, abs_tol: float = 0.05, rel_tol: float = 0.01) -> list[dict]:
    out = []
    for i, (g, w) in enumerate(zip(got, want)):
        j = next((j for j, (x, y) in enumerate(zip(g, w)) if x != y), None)
        if j is None:
            if len(g) != len(w):
                out.append({"req": i, "pos": min(len(g), len(w)), "near_tie": False, "why": "length"})
            continue
        probe = ref.generate([list(prompts[i]) + list(w[:j])],
                             SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True, embed=True))
        logits = ref.runner.model.compute_logits(ref.runner._last_hidden)[0].float()
        logits = logits[: ref.cfg.model_config.vocab_size]
        margin = float(logits[w[j]] - logits[g[j]])
        tol = max(abs_tol, rel_tol * float(logits.abs().max()))
        # a near tie: the reference's own logits at that position put the two tokens within tol; the
        # probe (the same prefix re-run alone) must pick one of them - bf16 logits tie exactly often
        # enough on random weights that a re-run's batch shape alone can flip an exact tie
        out.append({"req": i, "pos": j, "got": g[j], "want": w[j], "margin": round(margin, 4),
                    "tol": round(tol, 4), "probe": probe[0].output_token_ids[0],
                    "near_tie": margin <= tol and probe[0].output_token_ids[0] in (w[j], g[j])})
    return out


def assert_greedy_match(ref, prompts, got, want, **kw):
    div = first_divergences(ref, prompts, got, want, **kw)
    bad = [d for d in div if not d["near_tie"]]
    assert not bad, bad
    return div
