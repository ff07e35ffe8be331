import sys
sys.path.insert(0, ".")
from tests.test_lora import _make_adapter, _merged
from tests.test_engine import _prompts, greedy_reference, make_engine
from llmd_amd.engine.request import SamplingParams
for eager in (True, False):
    eng = make_engine(device="cuda", num_gpu_blocks=128, max_num_batched_tokens=256, model="small-llama",
                      max_num_seqs=8, enable_lora=True, max_loras=2, max_lora_rank=8, enforce_eager=eager)
    base = eng.runner.model
    d1 = _make_adapter(base, "/tmp/a1dbg", r=8, seed=3)
    eng.lora.load("a1", "/tmp/a1dbg")
    p = _prompts(5, [30], vocab=30000)[0]
    sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    print("eager", eager)
    r0 = eng.generate([p], sp, lora_ids=[0])[0]
    print(" base alone ", r0.output_token_ids)
    r, r0 = eng.generate([p, p], sp, lora_ids=[eng.lora.id_of("a1"), 0])
    print(" mixed      ", r.output_token_ids, r0.output_token_ids)
    r = eng.generate([p], sp, lora_ids=[eng.lora.id_of("a1")])[0]
    print(" adapter    ", r.output_token_ids)
    print(" ref adapter", greedy_reference(_merged(base, d1), p, 4))
    print(" ref base   ", greedy_reference(_merged(base, []), p, 4))
