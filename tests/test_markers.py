"""roctx markers: off by default (no library call), and with
LLMD_ROCTX on an engine step runs through nested ranges and kvx-style
start/stop ranges without error."""
import numpy as np

from llmd_amd.utils import markers


def test_markers_default_off_and_ranges_nest():
    assert not markers.enabled()
    with markers.range("x"):
        pass
    assert markers.start("y") == 0
    markers.stop(0)


def test_engine_step_with_roctx_enabled():
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    markers.set_enabled(True)
    try:
        rid = markers.start("llmd.kvx.pull test")
        markers.stop(rid)
        eng = LLMEngine(EngineConfig.create("tiny-llama", device="cpu", block_size=16, num_gpu_blocks=64,
                                            max_num_batched_tokens=64, max_num_seqs=4, max_model_len=256,
                                            enforce_eager=True))
        p = np.random.default_rng(0).integers(3, 500, size=20).tolist()
        r = eng.generate([p], SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))[0]
        assert len(r.output_token_ids) == 3
    finally:
        markers.set_enabled(False)
