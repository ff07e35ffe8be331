// Gated activations: out[T, F] = act(x[T, :F]) * x[T, F:].
//   mode 0: SiLU (SwiGLU, Llama/Qwen/DeepSeek)
//   mode 1: GELU-tanh (Gemma)
//   mode 2: gpt-oss clamped SwiGLU on an interleaved [g0,u0,g1,u1,...] layout:
//           g = min(g, limit); u = clamp(u, -limit, limit);
//           out = (u + 1) * g * sigmoid(alpha * g)
// Grid-stride over 16-byte chunks; 8 outputs per lane per step.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }
__device__ __forceinline__ float gelu_tanh(float g) {
  const float k = 0.7978845608028654f;  // sqrt(2/pi)
  return 0.5f * g * (1.f + tanhf(k * (g + 0.044715f * g * g * g)));
}

template <int MODE>
__global__ __launch_bounds__(NT) void act_kernel(uint16_t* __restrict__ out, int64_t os,
                                                 const uint16_t* __restrict__ x, int64_t xs,
                                                 int T, int F, float alpha, float limit) {
  const int cpr = F / 8;
  const int64_t total = (int64_t)T * cpr;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * NT) {
    const int t = (int)(i / cpr), c = (int)(i % cpr);
    const uint16_t* xr = x + (int64_t)t * xs;
    float g[8], u[8], o[8];
    if (MODE == 2) {
      // interleaved: 16 inputs -> 8 outputs
      float e[16];
      unpack8(*reinterpret_cast<const u32x4_t*>(xr + c * 16), e);
      unpack8(*reinterpret_cast<const u32x4_t*>(xr + c * 16 + 8), e + 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float gg = fminf(e[2 * j], limit);
        float uu = fminf(fmaxf(e[2 * j + 1], -limit), limit);
        o[j] = (uu + 1.f) * gg / (1.f + __expf(-alpha * gg));
      }
    } else {
      unpack8(*reinterpret_cast<const u32x4_t*>(xr + c * 8), g);
      unpack8(*reinterpret_cast<const u32x4_t*>(xr + F + c * 8), u);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (MODE == 0 ? silu(g[j]) : gelu_tanh(g[j])) * u[j];
    }
    *reinterpret_cast<u32x4_t*>(out + (int64_t)t * os + c * 8) = pack8(o);
  }
}

// Gated activation fused with dynamic per-row fp8 quantisation for the next
// W8A8 GEMM (SURVEY K07 "fused with per-token FP8 quant"): one workgroup per
// row; pass 1 computes the (bf16-rounded) activations and their amax, pass 2
// recomputes them from the L2-resident input, scales and writes e4m3fn.
template <int MODE>
__device__ __forceinline__ void act8(const uint16_t* xr, int F, int c, float alpha, float limit, float* o) {
  if (MODE == 2) {
    float e[16];
    unpack8(*reinterpret_cast<const u32x4_t*>(xr + c * 16), e);
    unpack8(*reinterpret_cast<const u32x4_t*>(xr + c * 16 + 8), e + 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gg = fminf(e[2 * j], limit);
      float uu = fminf(fmaxf(e[2 * j + 1], -limit), limit);
      o[j] = (uu + 1.f) * gg / (1.f + __expf(-alpha * gg));
    }
  } else {
    float g[8], u[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(xr + c * 8), g);
    unpack8(*reinterpret_cast<const u32x4_t*>(xr + F + c * 8), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (MODE == 0 ? silu(g[j]) : gelu_tanh(g[j])) * u[j];
  }
  unpack8(pack8(o), o);  // bf16 rounding, as the unfused path stores it
}

template <int MODE>
__global__ __launch_bounds__(NT) void act_quant_kernel(uint8_t* __restrict__ q, int64_t qs, float* __restrict__ scale,
                                                       const uint16_t* __restrict__ x, int64_t xs, int F, float alpha,
                                                       float limit) {
  __shared__ float red[NT / 64];
  const int64_t t = blockIdx.x;
  const uint16_t* xr = x + t * xs;
  const int cpr = F / 8;
  float amax = 0.f;
  for (int c = threadIdx.x; c < cpr; c += NT) {
    float o[8];
    act8<MODE>(xr, F, c, alpha, limit, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(o[j]));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red[i]);
  const float s = fmaxf(m / FP8_MAX, 1e-12f), is = 1.f / s;
  if (threadIdx.x == 0) scale[t] = s;
  u32x2_t* qr = reinterpret_cast<u32x2_t*>(q + t * qs);
  for (int c = threadIdx.x; c < cpr; c += NT) {
    float o[8];
    act8<MODE>(xr, F, c, alpha, limit, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] *= is;
    qr[c] = f32x8_to_fp8(o);
  }
}

}  // namespace

extern "C" void llmd_gated_act_quant(void* q, int64_t qs, float* scale, const void* x, int64_t xs, int T, int F,
                                     int mode, float alpha, float limit, hipStream_t st) {
  if (T == 0) return;
  dim3 g(T), b(NT);
  if (mode == 0)
    hipLaunchKernelGGL(act_quant_kernel<0>, g, b, 0, st, (uint8_t*)q, qs, scale, (const uint16_t*)x, xs, F, alpha,
                       limit);
  else if (mode == 1)
    hipLaunchKernelGGL(act_quant_kernel<1>, g, b, 0, st, (uint8_t*)q, qs, scale, (const uint16_t*)x, xs, F, alpha,
                       limit);
  else
    hipLaunchKernelGGL(act_quant_kernel<2>, g, b, 0, st, (uint8_t*)q, qs, scale, (const uint16_t*)x, xs, F, alpha,
                       limit);
}

extern "C" void llmd_gated_act(void* out, int64_t os, const void* x, int64_t xs, int T, int F,
                               int mode, float alpha, float limit, hipStream_t st) {
  if (T == 0) return;
  const int64_t chunks = (int64_t)T * (F / 8);
  int grid = (int)((chunks + NT - 1) / NT);
  if (grid > 2048) grid = 2048;
  dim3 g(grid), b(NT);
  if (mode == 0)
    hipLaunchKernelGGL(act_kernel<0>, g, b, 0, st, (uint16_t*)out, os, (const uint16_t*)x, xs,
                       T, F, alpha, limit);
  else if (mode == 1)
    hipLaunchKernelGGL(act_kernel<1>, g, b, 0, st, (uint16_t*)out, os, (const uint16_t*)x, xs,
                       T, F, alpha, limit);
  else
    hipLaunchKernelGGL(act_kernel<2>, g, b, 0, st, (uint16_t*)out, os, (const uint16_t*)x, xs,
                       T, F, alpha, limit);
}
