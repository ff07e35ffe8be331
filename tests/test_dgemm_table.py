"""Decode GEMM dispatch (CPU): table lookup buckets M up to the next measured
size, unmeasured shapes and CPU tensors stay on hipBLASLt / F.linear."""
import torch

from llmd_amd import ops
from llmd_amd.ops.dgemm_table import DGEMM_TABLE


def test_table_entries_are_wins_with_valid_plans():
    for (M, N, K), (plan, t_ours, t_blas) in DGEMM_TABLE.items():
        assert 1 <= M <= 64 and K % 256 == 0 and N % 4 == 0
        if plan is not None:
            rb, ns, occ = plan
            assert 1 <= rb <= 8 and 1 <= ns <= K // 256 and occ in (1, 2)
            assert t_ours < 0.95 * t_blas


def test_choice_buckets_and_unknown_shapes():
    assert ops.dgemm_choice(3, 4096, 4096) == DGEMM_TABLE[(8, 4096, 4096)][0]
    assert ops.dgemm_choice(20, 4096, 4096) is None  # 8B shapes: only M <= 8 measured as wins
    assert ops.dgemm_choice(1, 4096, 4096) == DGEMM_TABLE[(1, 4096, 4096)][0]
    assert ops.dgemm_choice(40, 8192, 28672) == DGEMM_TABLE[(48, 8192, 28672)][0]
    assert ops.dgemm_choice(64, 1234, 4096) is None
    assert ops.dgemm_choice(65, 4096, 4096) is None


def test_cpu_linear_is_plain():
    x = torch.randn(4, 256)
    w = torch.randn(64, 256)
    torch.testing.assert_close(ops.linear(x, w), x @ w.T)


def test_mgemm_table_entries_and_buckets():
    from llmd_amd.ops.mgemm_table import MGEMM_TABLE

    for (M, N, K), (plan, t_ours, t_other) in MGEMM_TABLE.items():
        assert M in (64, 96, 128, 192, 256) and K % 64 == 0 and N % 4 == 0
        if plan is not None:
            wrb, ns, stages = plan
            assert wrb in (1, 2, 4) and 1 <= ns <= K // 64 and stages in (3, 4)
            mb = 4 if M <= 64 else 6 if M <= 96 else 8 if M <= 128 else 12 if M <= 192 else 16
            assert stages * (64 * wrb * 128 + 16 * mb * 128) <= 160 * 1024  # LDS of the instantiation
            if mb > 8:  # the instantiated 192 / 256-row forms
                assert wrb == 1 or (wrb, stages) == (2, 3)
            assert t_ours < 0.95 * t_other
    # M 65..96 use the 96 row, 97..128 the 128 row, 129..192 the 192 row; unmeasured M/shape -> None
    assert ops.mgemm_choice(80, 5120, 8192) == MGEMM_TABLE[(96, 5120, 8192)][0]
    assert ops.mgemm_choice(100, 5120, 8192) == MGEMM_TABLE[(128, 5120, 8192)][0]
    assert ops.mgemm_choice(129, 5120, 8192) == MGEMM_TABLE[(192, 5120, 8192)][0]
    assert ops.mgemm_choice(257, 5120, 8192) is None
    assert ops.mgemm_choice(64, 1234, 4096) is None


def test_moe_tile_version_choice(monkeypatch):
    """Persistent expert-tile GEMM (moe8) choice: fp8 from 4 K-steps of 128, bf16 only for 4 .. 4096-deep
    K (gpt-oss 2880 yes, DeepSeek gate/up 7168 no), both switchable off."""
    assert ops.moe_tile_version("fp8", 2944) == 8 and ops.moe_tile_version("fp8", 7168) == 8
    assert ops.moe_tile_version("fp8", 384) == 4
    assert ops.moe_tile_version("bf16", 2880) == 8 and ops.moe_tile_version("bf16", 2048) == 8
    assert ops.moe_tile_version("bf16", 7168) == 4 and ops.moe_tile_version("bf16", 192) == 4
    monkeypatch.setattr(ops, "MOE_FP8_V8", False)
    monkeypatch.setattr(ops, "MOE_BF16_V8", False)
    assert ops.moe_tile_version("fp8", 2944) == 4 and ops.moe_tile_version("bf16", 2880) == 4
