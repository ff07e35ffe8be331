"""Shared-prefix (cascade) decode in the GPU engine: sequences that share a
cached 700-token prefix decode through the prefix kernel (hipGraph variant and
eager), and match an engine with the cascade off (GPU only)."""
import pytest

from greedy_check import first_divergences
from test_shared_prefix import _shared_prefix_run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,variant", [("tiny-llama", 1), ("small-llama", 3)])
@pytest.mark.parametrize("eager", [False, True])
def test_engine_shared_prefix_decode_gpu(monkeypatch, eager, model, variant):
    eng, prompts, got, used = _shared_prefix_run("cuda", monkeypatch, model, enforce_eager=eager)
    assert used
    assert eng.runner.casc_variant == variant
    if not eager:
        assert eng.runner.cgraphs, "no shared-prefix decode graphs captured"
    ref, _, want, used_off = _shared_prefix_run("cuda", monkeypatch, model, enforce_eager=eager,
                                                shared_prefix_decode=False)
    assert not used_off
    assert all(len(x) == 6 for x in got)
    # the prefix/suffix split sums the softmax in another order: a first divergence
    # must be a near-tie of the reference's logits (either sign; tiny random models
    # have near-flat logits, so the reference's own re-run may pick either token)
    div = first_divergences(ref, prompts, got, want)
    bad = [d for d in div if "margin" not in d or abs(d["margin"]) > d["tol"]]
    assert not bad, bad
