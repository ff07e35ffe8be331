"""Debug kernel build (device-side asserts in a debug build):
with LLMD_KERNEL_DEBUG=1 the ops load llmd_amd._C_debug (-O1 -g, LLMD_DCHECK
assertions compiled in) and the hot kernels still match the fp32 references on
valid inputs. Runs in a subprocess so the process-wide op library choice does
not leak into other tests. (A violated check traps the wave; that path is not
exercised on the shared GPU box.)"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import torch
from llmd_amd import ops
from llmd_amd.ops import reference as ref
C = ops.native()
assert C.__name__ == "llmd_amd._C_debug", C.__name__
torch.manual_seed(0)
dev = "cuda"
# paged decode + prefill on a small paged cache
Hq, Hkv, D, bs, ctx = 8, 2, 128, 64, 300
nb = 8
kc = torch.randn(nb, Hkv, bs, D, device=dev).bfloat16()
vc = torch.randn(nb, Hkv, bs, D, device=dev).bfloat16()
bt = torch.randperm(nb, device=dev)[:5].int().view(1, 5)
q = torch.randn(1, Hq * D, device=dev).bfloat16()
sl = torch.tensor([ctx], dtype=torch.int32, device=dev)
out = ops.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5)
want = ref.paged_decode(q, kc, vc, bt, sl, Hq, Hkv, D, D ** -0.5)
assert (out.float() - want.float()).abs().max().item() < 0.05
qp = torch.randn(ctx, Hq * D, device=dev).bfloat16()
qs = torch.tensor([0], dtype=torch.int32, device=dev)
ql = torch.tensor([ctx], dtype=torch.int32, device=dev)
outp = ops.paged_prefill(qp, kc, vc, bt, qs, ql, sl, Hq, Hkv, D, D ** -0.5)
wantp = ref.paged_prefill(qp, kc, vc, bt, qs, ql, sl, Hq, Hkv, D, D ** -0.5)
assert (outp.float() - wantp.float()).abs().max().item() < 0.05
# shared-prefix decode (both prefix kernels) + device-side split size: 4 sequences share 4 blocks
import numpy as np
nb2 = 24
kc2 = torch.randn(nb2, Hkv, bs, D, device=dev).bfloat16()
vc2 = torch.randn(nb2, Hkv, bs, D, device=dev).bfloat16()
rows = [[0, 1, 2, 3, 4 + 2 * i, 5 + 2 * i] for i in range(4)]
bt2 = np.array(rows, dtype=np.int32)
ln2 = np.array([300, 330, 383, 290], dtype=np.int32)
q2 = torch.randn(4, Hq * D, device=dev).bfloat16()
btd, lnd = torch.from_numpy(bt2).to(dev), torch.from_numpy(ln2).to(dev)
want2 = ref.paged_decode(q2, kc2, vc2, btd, lnd, Hq, Hkv, D, D ** -0.5)
for variant in (1, 3):
    plan = ops.shared_prefix_plan(bt2, ln2, bs, Hq // Hkv, Hkv, variant=variant, min_prefix=128, min_chunk=64)
    assert plan is not None and plan.items == 1, plan
    got2 = ops.paged_decode(q2, kc2, vc2, btd, lnd, Hq, Hkv, D, D ** -0.5, split=(256, 1),
                            cascade=ops.cascade_tensors(plan, dev),
                            split_dev=torch.tensor([128], dtype=torch.int32, device=dev))
    assert (got2.float() - want2.float()).abs().max().item() < 0.05, variant
# medium-M decode GEMM with split-K
x = torch.randn(96, 1024, device=dev).bfloat16()
w = (torch.randn(640, 1024, device=dev) * 0.05).bfloat16()
y = ops.mgemm(x, w, (2, 3, 3))
assert (y.float() - x.float() @ w.float().T).abs().max().item() < 0.05
torch.cuda.synchronize()
print("debug kernels ok")
'''


@pytest.mark.gpu
def test_debug_kernel_build_runs_hot_kernels():
    env = dict(os.environ, LLMD_KERNEL_DEBUG="1", LLMD_AUTOBUILD="0")
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "debug kernels ok" in r.stdout, r.stderr[-3000:]


def test_debug_build_flags():
    from llmd_amd import build

    src = open(os.path.join(ROOT, "llmd_amd/csrc/include/llmd_common.h")).read()
    assert "LLMD_DCHECK" in src and "LLMD_KERNEL_DEBUG" in src
    import inspect

    code = inspect.getsource(build.build_ops)
    assert "-DLLMD_KERNEL_DEBUG=1" in code and "_C_debug" in code
