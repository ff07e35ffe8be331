// Dynamic per-token FP8 quantisation (vLLM `dynamic_per_token_scaled_fp8_quant`).
//
// x [T, d] bf16 -> q [T, d] e4m3fn (OCP, gfx950) and scale [T] f32 with
// q = sat(x / scale), scale = max(|x_t|) / 448. One workgroup per row: pass 1
// reduces the row's amax (16-B loads, wave64 DPP reduction), pass 2 re-reads
// the row (L2/L1-resident after pass 1) and writes 8-B fp8 packets. This is the
// activation side of the FP8 linear (W8A8, per-channel weight scales), whose
// GEMM runs in hipBLASLt via torch._scaled_mm.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void quant_fp8_rows_kernel(const uint16_t* __restrict__ x, int64_t xs,
                                                            uint8_t* __restrict__ q, int64_t qs,
                                                            float* __restrict__ scale, int d, float floor_) {
  __shared__ float red[NT / 64];
  const int64_t t = blockIdx.x;
  const u32x4_t* xr = reinterpret_cast<const u32x4_t*>(x + t * xs);
  const int nc = d / 8;
  float amax = 0.f;
  for (int c = threadIdx.x; c < nc; c += NT) {
    float f[8];
    unpack8(xr[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(f[i]));
  }
  amax = wave_max(amax);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = amax;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red[i]);
  const float s = fmaxf(m / FP8_MAX, floor_);
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[t] = s;
  u32x2_t* qr = reinterpret_cast<u32x2_t*>(q + t * qs);
  for (int c = threadIdx.x; c < nc; c += NT) {
    float f[8];
    unpack8(xr[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] *= inv;
    qr[c] = f32x8_to_fp8(f);
  }
}

// Per (row, 128-element group) scales (DeepSeek / DeepGEMM activation format):
// 16 consecutive lanes own one group's 16 packets; the group amax is a 16-lane
// xor-shuffle reduction. s[t][g] = amax / 448.
// kp > d: q rows are kp bytes wide and columns [d, kp) are zero-filled (the K-padded operand of the
// grouped GEMM); row_limit (device scalar, nullable): rows at or past it are left untouched - the
// grouped GEMM's padded-slot rows beyond the last real expert tile, which it never reads.
// One wave per row (4 rows per 256-thread workgroup): a row of a few thousand columns is a few
// 8-column chunks per lane, and a 128-column group is 16 lanes, so the group amax is a 16-lane
// shuffle reduction inside the wave (a workgroup per row left most of its lanes idle).
__global__ __launch_bounds__(NT) void quant_fp8_groups_kernel(const uint16_t* __restrict__ x, int64_t xs,
                                                              uint8_t* __restrict__ q, int64_t qs,
                                                              float* __restrict__ scale, int64_t ss, int T,
                                                              int d, int kp, const int* __restrict__ row_limit,
                                                              float floor_) {
  const int64_t t = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T || (row_limit != nullptr && t >= *row_limit)) return;
  const u32x4_t* xr = reinterpret_cast<const u32x4_t*>(x + t * xs);
  u32x2_t* qr = reinterpret_cast<u32x2_t*>(q + t * qs);
  const int nc = d / 8;
  const int span = (nc + 15) / 16 * 16;  // whole 16-lane groups (a partial last group reads zeros)
  for (int c0 = 0; c0 < span; c0 += 64) {
    const int c = c0 + lane;
    const bool ok = c < nc;
    float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ok) unpack8(xr[c], f);
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a = fmaxf(a, fabsf(f[i]));
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
    const float sc = pow2_ceil(fmaxf(a / FP8_MAX, floor_));  // E8M0-exact (moe_gemm2_fp8_kernel)
    if (ok && (c & 15) == 0) scale[t * ss + c / 16] = sc;
    const float inv = 1.f / sc;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] *= inv;
    if (ok) qr[c] = f32x8_to_fp8(f);
  }
  for (int c = nc + lane; c < kp / 8; c += 64) qr[c] = u32x2_t{0u, 0u};
}

}  // namespace

extern "C" int llmd_quant_fp8_groups(const void* x, int64_t xs, void* q, int64_t qs, float* scale, int64_t ss,
                                     int T, int d, hipStream_t st) {
  if (T == 0) return 0;
  if (d % 8) return -1;
  hipLaunchKernelGGL(quant_fp8_groups_kernel, dim3((T + NT / 64 - 1) / (NT / 64)), dim3(NT), 0, st,
                     (const uint16_t*)x, xs, (uint8_t*)q, qs, scale, ss, T, d, d, (const int*)nullptr, 1e-12f);
  return (int)hipGetLastError();
}

// rows of kp >= d bytes (zeros past d), rows >= *row_limit skipped (row_limit nullable)
extern "C" int llmd_quant_fp8_groups_padded(const void* x, int64_t xs, void* q, int64_t qs, float* scale,
                                            int64_t ss, int T, int d, int kp, const int* row_limit,
                                            hipStream_t st) {
  if (T == 0) return 0;
  if (d % 8 || kp % 8 || kp < d || qs < kp) return -1;
  hipLaunchKernelGGL(quant_fp8_groups_kernel, dim3((T + NT / 64 - 1) / (NT / 64)), dim3(NT), 0, st,
                     (const uint16_t*)x, xs, (uint8_t*)q, qs, scale, ss, T, d, kp, row_limit, 1e-12f);
  return (int)hipGetLastError();
}

extern "C" int llmd_quant_fp8_rows(const void* x, int64_t xs, void* q, int64_t qs, float* scale, int T, int d,
                                   hipStream_t st) {
  if (T == 0) return 0;
  if (d % 8) return -1;
  hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3(T), dim3(NT), 0, st, (const uint16_t*)x, xs, (uint8_t*)q, qs,
                     scale, d, 1e-12f);
  return (int)hipGetLastError();
}
