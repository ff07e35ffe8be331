"""Shared-prefix (cascade) decode in the GPU engine: sequences that share a
cached 700-token prefix decode through the prefix kernel (hipGraph variant and
eager), and match an engine with the cascade off (GPU only)."""
import pytest

from greedy_check import first_divergences
from test_shared_prefix import _shared_prefix_run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,variant", [("tiny-llama", 1), ("small-llama", 3),
                                           ("tiny-gpt-oss", 3)])  # sliding-window layers + sinks
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


def test_graph_decode_splits_follow_context():
    """Decode graphs are planned for max_model_len (8k) but a step's splits are
    re-sized to its longest context at replay: graph and eager decode agree."""
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    prompts = [[(13 * i + j) % 30000 + 5 for j in range(200 + 150 * i)] for i in range(5)]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    outs = []
    for eager in (False, True):
        cfg = EngineConfig.create("small-llama", device="cuda", block_size=64, num_gpu_blocks=512,
                                  max_num_batched_tokens=4096, max_num_seqs=8, max_model_len=16384,
                                  cuda_graph_max_bs=8, enforce_eager=eager)
        eng = LLMEngine(cfg)
        if not eager:
            assert eng.runner.graph_plans[8][0] * eng.runner.graph_plans[8][1] >= eng.runner.max_model_len
        outs.append((eng, [r.output_token_ids for r in eng.generate(prompts, sp)]))
    (_, got), (ref, want) = outs
    div = first_divergences(ref, prompts, got, want)
    bad = [d for d in div if "margin" not in d or abs(d["margin"]) > d["tol"]]
    assert not bad, bad
