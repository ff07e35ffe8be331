// Energy per FLOP of the bf16 MFMA shapes under the package power cap: every wave keeps
// its A / B fragments and 4 independent accumulators in registers and issues MFMAs back to
// back (no memory traffic in the loop), one wave per SIMD on every CU. The harness
// (scripts/mfma_energy.py) loops a launch for seconds and samples clock + power.
//   shape 0: v_mfma_f32_16x16x32_bf16 (the prefill GEMM's), 1: v_mfma_f32_32x32x16_bf16
//   zero:    operands all zero (no data toggling) instead of random bits
// hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/probes/mfma_energy.hip -o scripts/probes/mfma_energy.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <int SHAPE>
__global__ __launch_bounds__(256, 1) void mfma_burn(float* out, int iters, int zero) {
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
  s16x8_t a[4], b[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // random bf16 in about [-2, 2] (sign, exponent 126..128, random mantissa), or zero
      const uint32_t h = hash32(tid * 64 + r * 8 + e);
      const short v = (short)((h & 0x8000u) | (0x3f00u + (h & 0x017fu)));
      a[r][e] = zero ? 0 : v;
      b[r][e] = zero ? 0 : (short)(v ^ 0x0055);
    }
  float sink = 0.f;
  if constexpr (SHAPE == 0) {
    f32x4_t c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r], b[r], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r], b[(r + 1) & 3], c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(r + 2) & 3], b[r], c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(r + 3) & 3], b[(r + 2) & 3], c3, 0, 0, 0);
      }
    }
    sink = c0[0] + c1[1] + c2[2] + c3[3];
  } else {
    // 32x32x16 takes 8 bf16 per lane of A / B too (k 16 = 2 x 8 across the lane halves)
    f32x16_t c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[r], b[r], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[r + 1], b[(r + 3) & 3], c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[r + 2], b[r + 1], c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(r + 3) & 3], b[r + 2], c3, 0, 0, 0);
      }
    }
    sink = c0[0] + c1[5] + c2[9] + c3[13];
  }
  out[tid] = sink;
}

extern "C" int mfma_burn_launch(float* out, int shape, int zero, int iters, int blocks) {
  if (shape == 0)
    hipLaunchKernelGGL(mfma_burn<0>, dim3(blocks), dim3(256), 0, 0, out, iters, zero);
  else
    hipLaunchKernelGGL(mfma_burn<1>, dim3(blocks), dim3(256), 0, 0, out, iters, zero);
  return (int)hipGetLastError();
}
