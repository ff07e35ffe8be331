"""New model families end to end on the GPU engine (HIP kernels + hipGraph
decode): multimodal tiny-vl (vision tower + placeholder splice), Qwen3-MoE
style tiny-moe, and fp8 W8A8 + fp8 KV on tiny-llama."""
import pytest
import torch

from llmd_amd.engine.config import EngineConfig
from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import SamplingParams

pytestmark = pytest.mark.gpu


def _eng(model, **kw):
    cfg = EngineConfig.create(model, device="cuda", block_size=64, num_gpu_blocks=64, max_num_batched_tokens=256,
                              max_num_seqs=4, max_model_len=1024, cuda_graph_max_bs=4, **kw)
    return LLMEngine(cfg)


def test_moe_llama_gpu_matches_eager():
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    prompts = [list(range(5, 60)), [11] * 30]
    a = [r.output_token_ids for r in _eng("tiny-moe").generate(prompts, sp)]
    b = [r.output_token_ids for r in _eng("tiny-moe", enforce_eager=True).generate(prompts, sp)]
    assert a == b and all(len(x) == 6 for x in a)


def test_vl_gpu_chunked_image():
    import io

    from PIL import Image

    from llmd_amd.models.vision import MMInput, mm_hash

    arr = (torch.rand(112, 84, 3) * 255).to(torch.uint8).numpy()
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    img = buf.getvalue()
    outs = []
    for mbt in (256, 16):
        cfg = EngineConfig.create("tiny-vl", device="cuda", block_size=64, num_gpu_blocks=64,
                                  max_num_batched_tokens=mbt, max_num_seqs=4, max_model_len=1024,
                                  enable_prefix_caching=False, cuda_graph_max_bs=4)
        eng = LLMEngine(cfg)
        emb = eng.runner.model.encode_image(img)
        n = emb.shape[0]
        ids = list(range(10, 15)) + [cfg.model_config.image_token_id] * n + list(range(15, 40))
        r = eng.add_request("a", ids, SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True),
                            mm_inputs=[MMInput(5, n, mm_hash(img), emb)])
        while eng.has_unfinished():
            eng.step()
        outs.append(r.output_token_ids)
    assert outs[0] == outs[1] and len(outs[0]) == 5


def test_fp8_engine_gpu():
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    eng = _eng("tiny-llama", quantization="fp8", kv_cache_dtype="fp8")
    assert eng.runner.kv.dtype == torch.float8_e4m3fn
    rs = eng.generate([list(range(3, 90)), [5] * 40], sp)
    assert all(len(r.output_token_ids) == 8 for r in rs)
