// Multi-LoRA batched GEMV (the punica/BGMV role): every token row
// carries an adapter slot index (0 = no adapter) and gets
//   y[t] += B[slot] @ (A[slot] @ x[t])
// with the adapters of all resident slots stacked: A [S, R, in], B [S, out, R]
// (scaling pre-folded into B). Graph-capturable: slots live on the device.
//
// shrink: one workgroup per (token, 16-rank group); the token's x row is
//   staged in LDS once (<= 64 KiB for in <= 32768), each wave computes 4 ranks
//   as full-row dot products with 16-B loads of A and a wave reduction.
// expand: one workgroup per (token, 256-output chunk); each lane owns one
//   output row and dots its R contiguous B entries with h[t] held in LDS.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void lora_shrink_kernel(const uint16_t* __restrict__ x, int64_t x_stride,
                                                         const uint16_t* __restrict__ A, int R, int in,
                                                         const int* __restrict__ slot, float* __restrict__ h) {
  const int t = blockIdx.x, rg = blockIdx.y;
  const int s = slot[t];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (s <= 0) {
    if (threadIdx.x < 16 && rg * 16 + threadIdx.x < R) h[(int64_t)t * R + rg * 16 + threadIdx.x] = 0.f;
    return;
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem);
  const uint16_t* xr = x + (int64_t)t * x_stride;
  for (int i = threadIdx.x; i < in / 8; i += NT)
    reinterpret_cast<u32x4_t*>(xs)[i] = reinterpret_cast<const u32x4_t*>(xr)[i];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = rg * 16 + w * 4 + j;
    if (r >= R) break;
    const uint16_t* ar = A + ((int64_t)s * R + r) * in;
    float acc = 0.f;
    for (int i = lane; i < in / 8; i += 64) {
      const bf16x8_t av = __builtin_bit_cast(bf16x8_t, reinterpret_cast<const u32x4_t*>(ar)[i]);
      const bf16x8_t xv = __builtin_bit_cast(bf16x8_t, reinterpret_cast<const u32x4_t*>(xs)[i]);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += (float)av[k] * (float)xv[k];
    }
    acc = wave_sum(acc);
    if (lane == 0) h[(int64_t)t * R + r] = acc;
  }
}

__global__ __launch_bounds__(NT) void lora_expand_kernel(const float* __restrict__ h, const uint16_t* __restrict__ B,
                                                         int R, int out, const int* __restrict__ slot,
                                                         uint16_t* __restrict__ y, int64_t y_stride) {
  const int t = blockIdx.x;
  const int s = slot[t];
  if (s <= 0) return;
  __shared__ float hs[128];
  if (threadIdx.x < R) hs[threadIdx.x] = h[(int64_t)t * R + threadIdx.x];
  __syncthreads();
  const int o = blockIdx.y * NT + threadIdx.x;
  if (o >= out) return;
  const uint16_t* br = B + ((int64_t)s * out + o) * R;
  float acc = 0.f;
  for (int r = 0; r < R; ++r) acc += bf2f(br[r]) * hs[r];
  uint16_t* yr = y + (int64_t)t * y_stride + o;
  *yr = f2bf(bf2f(*yr) + acc);
}

}  // namespace

extern "C" int llmd_lora_bgmv(const void* x, int64_t x_stride, const void* A, const void* B, int T, int R, int in,
                              int out, const int* slot, float* h, void* y, int64_t y_stride, hipStream_t st) {
  if (T == 0) return 0;
  if (R > 128 || in % 8 != 0 || in > 32768) return -1;
  hipLaunchKernelGGL(lora_shrink_kernel, dim3(T, (R + 15) / 16), dim3(NT), in * 2, st, (const uint16_t*)x, x_stride,
                     (const uint16_t*)A, R, in, slot, h);
  hipLaunchKernelGGL(lora_expand_kernel, dim3(T, (out + NT - 1) / NT), dim3(NT), 0, st, h, (const uint16_t*)B, R,
                     out, slot, (uint16_t*)y, y_stride);
  return (int)hipGetLastError();
}
