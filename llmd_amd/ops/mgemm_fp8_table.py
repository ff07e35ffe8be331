"""fp8 W8A8 medium-M decode GEMM dispatch table (csrc/ops/mgemm.hip F8 form;
scripts/sweep_mgemm_fp8.py on 1x MI355X, weights cold in HBM).

(M, N, K) -> (plan (wrb, nsplit, stages) or None, our us, hipBLASLt scaled-GEMM us
with the TunableOp table). A plan is listed only where the kernel beat
torch._scaled_mm by >= 5 %.
"""

MGEMM_FP8_TABLE = {
    (64, 10240, 8192): ((2, 3, 3), 24.1, 27.7),
    (96, 10240, 8192): ((2, 3, 3), 27.9, 30.2),
    (128, 10240, 8192): (None, 34.1, 33.1),
    (64, 8192, 8192): ((1, 2, 4), 19.9, 25.5),
    (96, 8192, 8192): ((1, 2, 3), 23.4, 24.7),
    (128, 8192, 8192): (None, 26.4, 25.4),
    (64, 57344, 8192): ((4, 1, 3), 87.1, 104.4),
    (96, 57344, 8192): ((4, 1, 3), 98.4, 106.9),
    (128, 57344, 8192): (None, 114.9, 105.7),
    (64, 8192, 28672): ((1, 2, 4), 51.3, 62.1),
    (96, 8192, 28672): ((1, 4, 3), 62.1, 89.1),
    (128, 8192, 28672): (None, 72.1, 73.4),
}
