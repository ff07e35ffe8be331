import sys
import torch
sys.path.insert(0, ".")
from tests.test_lora import _make_adapter
from tests.test_engine import make_engine
from llmd_amd import ops
from llmd_amd.ops import reference as ref
eng = make_engine(device="cuda", num_gpu_blocks=128, max_num_batched_tokens=256, model="small-llama",
                  max_num_seqs=8, enable_lora=True, max_loras=2, max_lora_rank=8, enforce_eager=True)
base = eng.runner.model
d1 = _make_adapter(base, "/tmp/a1dbg", r=8, seed=3)
eng.lora.load("a1", "/tmp/a1dbg")
T = 30
eng.lora.set_tokens([1] * T)
torch.cuda.synchronize()
print("slots", eng.lora.slot_idx[:T].tolist()[:5])
L0 = base.layers[0]
x = torch.randn(T, 1024, device="cuda").bfloat16()
for name, mod, key in (("qkv", L0.qkv, None), ("o", L0.o_proj, "o"), ("gate_up", L0.mlp.gate_up, None),
                       ("down", L0.mlp.down, "down")):
    xin = x if mod.in_f == 1024 else torch.randn(T, mod.in_f, device="cuda").bfloat16()
    y = mod(xin)
    lo = mod.lora
    mod.lora = None
    y0 = mod(xin)
    mod.lora = lo
    yr = ref.lora_bgmv(y0.clone(), xin, lo.A, lo.B, eng.lora.slot_idx[:T])
    print(name, "engine-vs-ref", (y.float() - yr.float()).abs().max().item(), "delta", (yr.float() - y0.float()).abs().max().item())
