"""MXFP4 experts (OCP MX: e2m1 codes + E8M0 scale per 32 elements - gpt-oss's checkpoint format):
the quantiser's format contract on CPU, and on the GPU the persistent expert-tile kernel
(csrc/ops/moe8.hip moe_gemm8_mxfp4_kernel) against the fp32 oracle of the same quantised operands -
one GEMM on its own (gathered rows, expert bias, gpt-oss activation) and the whole layer at gpt-oss
widths (K padded 2880 -> 2944, partial column tiles), prefill- and decode-sized steps."""
import math

import pytest
import torch

from llmd_amd import ops


def test_mxfp4_codes_scales_and_packing():
    w = torch.tensor([0.5, -1.0, 6.0, -6.0, 3.0, 0.0, 1.5, -4.0] * 4).view(1, 1, 32)
    q, s = ops.quant_mxfp4_weight(w)
    assert q.shape == (1, 1, 16) and s.shape == (1, 1, 1) and int(s) == 127
    assert int(q[0, 0, 0]) == 0x1 | (0xA << 4)  # 0.5 = code 1 (low nibble), -1.0 = 8 | 2 (high nibble)
    assert torch.equal(ops.dequant_mxfp4_weight(q, s), w)
    torch.manual_seed(0)
    w = torch.randn(2, 4, 128) * 0.03
    q, s = ops.quant_mxfp4_weight(w)
    d = ops.dequant_mxfp4_weight(q, s)
    amax = w.view(2, 4, 4, 32).abs().amax(-1, keepdim=True)
    # every block's largest magnitude maps into (3, 6] * scale; error <= half the widest e2m1 step (1) * scale
    scale = torch.exp2(s.float() - 127)[..., None]
    assert ((w.view(2, 4, 4, 32) / scale).abs().amax(-1) <= 6.0 + 1e-6).all()
    assert ((d - w).view(2, 4, 4, 32).abs() <= scale * 1.0 + 1e-9).all()
    assert (amax > 0).all()


def test_moe_experts_mxfp4_cpu_reference_runs():
    torch.manual_seed(1)
    T, E, k, d, F = 6, 4, 2, 256, 128
    x = torch.randn(T, d, dtype=torch.bfloat16)
    w1q, w1s = ops.quant_mxfp4_weight(torch.randn(E, 2 * F, d) * 0.05)
    w2q, w2s = ops.quant_mxfp4_weight(torch.randn(E, d, F) * 0.05)
    ids, wts = ops.moe_topk(torch.randn(T, E), k, scoring=0)
    y = ops.moe_experts_mxfp4(x, ids, wts, w1q, w1s, w2q, w2s, act=2)
    assert y.shape == (T, d) and torch.isfinite(y.float()).all()


def _oracle_rows(xq, xs, wq, ws, bias, sorted_ids, tile_e, tile, k, mode):
    K = xq.shape[1]
    xd = xq.float() * xs.repeat_interleave(128, 1)[:, :K]
    wd = ops.dequant_mxfp4_weight(wq, ws).float()
    sid = sorted_ids.long()
    live = sid >= 0
    te = tile_e.long().repeat_interleave(tile)[:sid.numel()]
    ref = torch.zeros(sid.numel(), wq.shape[1], device=xq.device)
    for e in range(wq.shape[0]):
        rows = live & (te == e)
        if rows.any():
            ref[rows] = xd[sid[rows] // k] @ wd[e].T + bias[e].float()
    if mode == 1:
        g, u = ref[:, 0::2].clamp(max=7.0), ref[:, 1::2].clamp(-7.0, 7.0)
        ref = (u + 1) * g * torch.sigmoid(1.702 * g)
    return ref, live


@pytest.mark.gpu
@pytest.mark.parametrize("mode,tile,stages,K", [(0, 256, 2, 2944), (1, 256, 3, 2944), (1, 192, 2, 2944),
                                                (0, 192, 3, 2944), (1, 256, 2, 512), (0, 192, 3, 512),
                                                (0, 64, 2, 2944), (1, 64, 2, 2944), (1, 64, 3, 512)])
def test_moe_gemm8_mxfp4_matches_fp32(mode, tile, stages, K, monkeypatch):
    """stages: LDS K-step buffers of the stream (2 = default, 3 opt-in); K = 512 is the shortest K loop
    (4 steps: every step is a peeled tile-transition phase); each case runs both weight layouts."""
    monkeypatch.setenv("LLMD_MXFP4_STAGES", str(stages))
    torch.manual_seed(5)
    dev = "cuda"
    C = ops.native()
    T, E, k = 400, 8, 4
    N = 5760 if mode == 1 else 2880
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    xq, xs = ops._quant_groups_padded(x, K)
    wq, ws = ops.quant_mxfp4_weight(torch.randn(E, N, K, device=dev) * 0.03)
    bias = torch.randn(E, N, device=dev, dtype=torch.bfloat16) * 0.1
    ids, _ = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    n = T * k
    max_p = ((n + E * (tile - 1)) + tile - 1) // tile * tile
    sorted_ids = torch.empty(max_p, dtype=torch.int32, device=dev)
    tile_e = torch.empty(max_p // tile, dtype=torch.int32, device=dev)
    offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
    total = torch.empty(1, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    C.moe_align(ids.contiguous().view(-1).to(torch.int32), E, sorted_ids, tile_e, offs, total, inv, tile)
    ref, live = _oracle_rows(xq, xs, wq, ws, bias, sorted_ids, tile_e, tile, k, mode)
    m = ref[live].abs().max().item()
    # both weight layouts: the packed standard order and K-step major (ops.mxfp4_kernel_layout)
    for w, sc in ((wq, ws), (ops.mxfp4_kernel_layout(wq), ops.mxfp4_scales_kernel_layout(ws))):
        y = torch.full((max_p, N // 2 if mode == 1 else N), 7.0, device=dev, dtype=torch.bfloat16)
        C.moe_gemm8_mxfp4(xq, xs, k, sorted_ids, tile_e, w, sc, y, mode, 2, 1.702, 7.0, False, bias, tile, total)
        torch.cuda.synchronize()
        got = y.float()
        assert (got[live] - ref[live]).abs().max().item() < 0.01 * m + 1e-2, w.dim()
        assert (got[~live] == 7.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [5, 64, 700])
def test_moe_experts_mxfp4_gpu_vs_cpu(T):
    torch.manual_seed(3)
    dev = "cuda"
    E, k, d, F = 16, 4, 2880, 2880
    c128 = lambda n: (n + 127) // 128 * 128  # noqa: E731
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w1 = ops.pad_mxfp4_k(torch.randn(E, 2 * F, d, device=dev) * 0.03, c128(d))
    w2 = ops.pad_mxfp4_k(torch.randn(E, d, F, device=dev) * 0.03, c128(F))
    w1q, w1s = ops.quant_mxfp4_weight(w1)
    w2q, w2s = ops.quant_mxfp4_weight(w2)
    w1q, w2q = ops.mxfp4_kernel_layout(w1q), ops.mxfp4_kernel_layout(w2q)  # the layout the model stores
    w1s, w2s = ops.mxfp4_scales_kernel_layout(w1s), ops.mxfp4_scales_kernel_layout(w2s)
    b1 = torch.randn(E, 2 * F, device=dev, dtype=torch.bfloat16) * 0.1
    b2 = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.1
    ids, wts = ops.moe_topk(torch.randn(T, E, device=dev), k, scoring=0)
    y = ops.moe_experts_mxfp4(x, ids, wts, w1q, w1s, w2q, w2s, 2, b1=b1, b2=b2)
    r = ops.moe_experts_mxfp4(x.cpu(), ids.cpu(), wts.cpu(), w1q.cpu(), w1s.cpu(), w2q.cpu(), w2s.cpu(), 2,
                              b1=b1.cpu(), b2=b2.cpu())
    m = r.float().abs().max().item()
    assert torch.isfinite(y.float()).all()
    assert (y.float().cpu() - r.float()).abs().max().item() < 0.06 * m + 1e-3


def test_load_mxfp4_checkpoint_experts_lossless(tmp_path):
    """gpt-oss checkpoints ship experts as MXFP4 ``*_blocks`` [E, out, K/32, 16] + ``*_scales`` [E, out, K/32]:
    the loader dequantises them, and ``--quantization mxfp4`` re-quantises them to exactly the checkpoint's values."""
    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.models import build_model
    from llmd_amd.models.loader import export_hf, load_weights, save_safetensors

    kw = dict(device="cpu", block_size=16, num_gpu_blocks=64, max_num_batched_tokens=64, max_num_seqs=4,
              max_model_len=256, enforce_eager=True)
    mc = EngineConfig.create("tiny-gpt-oss", **kw).model_config
    torch.manual_seed(0)
    tensors = export_hf(build_model(mc, device="cpu", max_pos=300))
    packed = {}
    for name in [n for n in tensors if n.endswith(("mlp.experts.gate_up_proj", "mlp.experts.down_proj"))]:
        w = tensors.pop(name).transpose(1, 2).float()  # HF [E, in, out] -> [E, out, in]
        q, s = ops.quant_mxfp4_weight(w)
        E, N, K2 = q.shape
        tensors[name + "_blocks"] = q.view(E, N, K2 // 16, 16)
        tensors[name + "_scales"] = s
        packed[name] = (q, s)
    assert packed
    path = str(tmp_path / "mx.safetensors")
    save_safetensors(tensors, path)

    m2 = build_model(mc, device="cpu", max_pos=300)
    load_weights(m2, path)
    eng = LLMEngine(EngineConfig.create("tiny-gpt-oss", load_format="safetensors", weights_path=path,
                                        quantization="mxfp4", **kw))
    by_name2 = {n: p for n, p, _, _ in m2.weight_specs()}
    by_name_q = {n: (p, own) for n, p, _, own in eng.runner.model.weight_specs()}
    mods = {id(getattr(m, a)): (m, a) for m in eng.runner.model.modules() for a in ("w1", "w2")
            if isinstance(getattr(m, a, None), torch.Tensor)}
    for name, (q, s) in packed.items():
        key = name if name in by_name2 else "model." + name
        assert torch.equal(by_name2[key], ops.dequant_mxfp4_weight(q, s).to(torch.bfloat16))
        pq = by_name_q[key][0]
        m, a = mods[id(pq)]
        assert pq.dtype == torch.uint8
        # the same values (a block whose largest code is 3 may come back as 6 at half the scale)
        K = 2 * q.shape[2]
        assert pq.dim() == 4  # stored K-step major for the tile kernel
        got = ops.dequant_mxfp4_weight(ops.mxfp4_std_layout(pq),
                                       ops.mxfp4_scales_std_layout(getattr(m, a + "_scale")))[..., :K]
        assert torch.equal(got, ops.dequant_mxfp4_weight(q, s))
    out = eng.generate([[5, 6, 7, 8, 9]], __import__("llmd_amd.engine.request", fromlist=["SamplingParams"])
                       .SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    assert len(out[0].output_token_ids) == 3
