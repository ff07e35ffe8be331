// RMSNorm and fused residual-add + RMSNorm.
//
// One workgroup (256 threads = 4 waves) per row. Each lane owns VPT 16-byte
// chunks (8 bf16) of the row, kept in registers between the reduction and the
// normalisation so the row is read from HBM exactly once. The fused variant
// writes the updated residual and the normalised activations in the same pass
// (vLLM `fused_add_rms_norm` semantics, reference: vLLM `_C` ops listed in
// docker/scripts/cuda/runtime/install-vllm.sh).
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

template <int VPT, bool FUSED_ADD>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(
    uint16_t* __restrict__ out, int64_t out_stride,
    uint16_t* __restrict__ x, int64_t x_stride,
    uint16_t* __restrict__ residual, int64_t res_stride,
    const uint16_t* __restrict__ w, int d, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const int nchunk = d >> 3;
  uint16_t* xr = x + (int64_t)row * x_stride;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
      u32x4_t a = *reinterpret_cast<const u32x4_t*>(xr + ci * 8);
      unpack8(a, v[c]);
      if constexpr (FUSED_ADD) {
        uint16_t* rr = residual + (int64_t)row * res_stride;
        u32x4_t r = *reinterpret_cast<const u32x4_t*>(rr + ci * 8);
        float rf[8];
        unpack8(r, rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += rf[j];
        // round the residual to bf16 once, and normalise the rounded value
        u32x4_t p = pack8(v[c]);
        *reinterpret_cast<u32x4_t*>(rr + ci * 8) = p;
        unpack8(p, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = block_sum<NT>(ss, red);
  const float inv = rsqrtf(ss / (float)d + eps);
  uint16_t* orow = (FUSED_ADD ? xr : out + (int64_t)row * out_stride);
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
      u32x4_t wa = *reinterpret_cast<const u32x4_t*>(w + ci * 8);
      float wf[8];
      unpack8(wa, wf);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * inv * wf[j];
      *reinterpret_cast<u32x4_t*>(orow + ci * 8) = pack8(o);
    }
  }
}

template <bool FUSED>
void launch(uint16_t* out, int64_t os, uint16_t* x, int64_t xs, uint16_t* res, int64_t rs,
            const uint16_t* w, int rows, int d, float eps, hipStream_t st) {
  const int nchunk = d / 8;
  const int vpt = (nchunk + NT - 1) / NT;
  dim3 g(rows), b(NT);
#define L(V)                                                                                 \
  hipLaunchKernelGGL((rmsnorm_kernel<V, FUSED>), g, b, 0, st, out, os, x, xs, res, rs, w, d, \
                     eps)
  if (vpt <= 1) L(1);
  else if (vpt <= 2) L(2);
  else if (vpt <= 4) L(4);
  else if (vpt <= 8) L(8);
  else L(16);
#undef L
}

// RMSNorm (optionally fused with the residual add) emitting fp8 e4m3fn with a
// per-row dynamic scale for the next W8A8 GEMM (SURVEY K05 "+ optional FP8
// quant"): the normalised row (rounded to bf16, as the unfused path would
// store it) stays in registers, a second block reduction takes its amax, and
// 8-B fp8 packets are written - no bf16 activation round trip through HBM.
template <int VPT, bool FUSED_ADD>
__global__ __launch_bounds__(NT) void rmsnorm_quant_kernel(
    uint8_t* __restrict__ q, int64_t q_stride, float* __restrict__ scale,
    const uint16_t* __restrict__ x, int64_t x_stride,
    uint16_t* __restrict__ residual, int64_t res_stride,
    const uint16_t* __restrict__ w, int d, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const int nchunk = d >> 3;
  const uint16_t* xr = x + (int64_t)row * x_stride;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
      u32x4_t a = *reinterpret_cast<const u32x4_t*>(xr + ci * 8);
      unpack8(a, v[c]);
      if constexpr (FUSED_ADD) {
        uint16_t* rr = residual + (int64_t)row * res_stride;
        u32x4_t r = *reinterpret_cast<const u32x4_t*>(rr + ci * 8);
        float rf[8];
        unpack8(r, rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += rf[j];
        u32x4_t p = pack8(v[c]);
        *reinterpret_cast<u32x4_t*>(rr + ci * 8) = p;
        unpack8(p, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = block_sum<NT>(ss, red);
  const float inv = rsqrtf(ss / (float)d + eps);
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
      u32x4_t wa = *reinterpret_cast<const u32x4_t*>(w + ci * 8);
      float wf[8];
      unpack8(wa, wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = v[c][j] * inv * wf[j];
      unpack8(pack8(v[c]), v[c]);  // bf16 rounding of the normalised value
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[c][j]));
    }
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red[i]);
  const float s = fmaxf(m / FP8_MAX, 1e-12f);
  const float is = 1.f / s;
  if (threadIdx.x == 0) scale[row] = s;
  u32x2_t* qr = reinterpret_cast<u32x2_t*>(q + (int64_t)row * q_stride);
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] *= is;
      qr[ci] = f32x8_to_fp8(v[c]);
    }
  }
}

template <bool FUSED>
void launch_q(uint8_t* q, int64_t qs, float* scale, const uint16_t* x, int64_t xs, uint16_t* res, int64_t rs,
              const uint16_t* w, int rows, int d, float eps, hipStream_t st) {
  const int nchunk = d / 8;
  const int vpt = (nchunk + NT - 1) / NT;
  dim3 g(rows), b(NT);
#define L(V) \
  hipLaunchKernelGGL((rmsnorm_quant_kernel<V, FUSED>), g, b, 0, st, q, qs, scale, x, xs, res, rs, w, d, eps)
  if (vpt <= 1) L(1);
  else if (vpt <= 2) L(2);
  else if (vpt <= 4) L(4);
  else if (vpt <= 8) L(8);
  else L(16);
#undef L
}

// LayerNorm with weight and bias (OPT-family decoders), optionally fused with
// the residual add, same one-row-per-workgroup register-resident layout: the
// mean and then the centred sum of squares are two block reductions over the
// values already in registers (no second HBM read, no E[x^2]-E[x]^2 cancellation).
template <int VPT, bool FUSED_ADD>
__global__ __launch_bounds__(NT) void layernorm_kernel(
    uint16_t* __restrict__ out, int64_t out_stride,
    uint16_t* __restrict__ x, int64_t x_stride,
    uint16_t* __restrict__ residual, int64_t res_stride,
    const uint16_t* __restrict__ w, const uint16_t* __restrict__ b, int d, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const int nchunk = d >> 3;
  uint16_t* xr = x + (int64_t)row * x_stride;
  float v[VPT][8];
  float s1 = 0.f;
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
      u32x4_t a = *reinterpret_cast<const u32x4_t*>(xr + ci * 8);
      unpack8(a, v[c]);
      if constexpr (FUSED_ADD) {
        uint16_t* rr = residual + (int64_t)row * res_stride;
        u32x4_t r = *reinterpret_cast<const u32x4_t*>(rr + ci * 8);
        float rf[8];
        unpack8(r, rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += rf[j];
        u32x4_t p = pack8(v[c]);
        *reinterpret_cast<u32x4_t*>(rr + ci * 8) = p;
        unpack8(p, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s1 += v[c][j];
    }
  }
  const float mean = block_sum<NT>(s1, red) / (float)d;  // block_sum ends with a barrier: red is free again
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = v[c][j] - mean;
        s2 += t * t;
      }
    }
  }
  const float inv = rsqrtf(block_sum<NT>(s2, red) / (float)d + eps);
  uint16_t* orow = (FUSED_ADD ? xr : out + (int64_t)row * out_stride);
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int ci = threadIdx.x + c * NT;
    if (ci < nchunk) {
      float wf[8], bf[8], o[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(w + ci * 8), wf);
      unpack8(*reinterpret_cast<const u32x4_t*>(b + ci * 8), bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * inv * wf[j] + bf[j];
      *reinterpret_cast<u32x4_t*>(orow + ci * 8) = pack8(o);
    }
  }
}

template <bool FUSED>
void launch_ln(uint16_t* out, int64_t os, uint16_t* x, int64_t xs, uint16_t* res, int64_t rs, const uint16_t* w,
               const uint16_t* b, int rows, int d, float eps, hipStream_t st) {
  const int nchunk = d / 8;
  const int vpt = (nchunk + NT - 1) / NT;
  dim3 g(rows), blk(NT);
#define L(V) \
  hipLaunchKernelGGL((layernorm_kernel<V, FUSED>), g, blk, 0, st, out, os, x, xs, res, rs, w, b, d, eps)
  if (vpt <= 1) L(1);
  else if (vpt <= 2) L(2);
  else if (vpt <= 4) L(4);
  else if (vpt <= 8) L(8);
  else L(16);
#undef L
}

// Qwen3 per-head RMSNorm of q and k, in place inside the fused QKV output
// (qkv[T, (Hq + 2 Hkv) * D]; heads [0, Hq) use qw, [Hq, Hq + Hkv) use kw, V is
// untouched). One wave per head: each lane owns E = D / 64 consecutive
// elements, the sum of squares is a 64-lane shuffle reduction, and the head is
// read and written once - no strided copies out of / back into the QKV buffer.
template <int E>
__global__ __launch_bounds__(NT) void qk_rmsnorm_kernel(uint16_t* __restrict__ qkv, int64_t stride,
                                                        const uint16_t* __restrict__ qw,
                                                        const uint16_t* __restrict__ kw, int Hq, int Hkv,
                                                        float eps) {
  constexpr int D = 64 * E;
  const int t = blockIdx.x;
  const int h = blockIdx.y * (NT / 64) + (threadIdx.x >> 6);
  if (h >= Hq + Hkv) return;  // whole wave exits together
  const int lane = threadIdx.x & 63;
  uint16_t* hp = qkv + (int64_t)t * stride + (int64_t)h * D + lane * E;
  const uint16_t* w = (h < Hq ? qw : kw) + lane * E;
  float v[E];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    v[j] = bf2f(hp[j]);
    ss += v[j] * v[j];
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int j = 0; j < E; ++j) hp[j] = f2bf(v[j] * inv * bf2f(w[j]));
}

}  // namespace

extern "C" {
// qkv[:, :Hq*D] = rmsnorm_head(q) * qw, qkv[:, Hq*D:(Hq+Hkv)*D] = rmsnorm_head(k) * kw (in place)
int llmd_qk_rms_norm(void* qkv, int64_t stride, const void* qw, const void* kw, int T, int Hq, int Hkv, int D,
                     float eps, hipStream_t st) {
  if (T == 0) return 0;
  dim3 g(T, (Hq + Hkv + NT / 64 - 1) / (NT / 64)), b(NT);
#define L(E)                                                                                             \
  hipLaunchKernelGGL((qk_rmsnorm_kernel<E>), g, b, 0, st, (uint16_t*)qkv, stride, (const uint16_t*)qw, \
                     (const uint16_t*)kw, Hq, Hkv, eps)
  if (D == 64) L(1);
  else if (D == 128) L(2);
  else if (D == 256) L(4);
  else return -1;
#undef L
  return 0;
}

// out = layernorm(x) * w + b; with residual: residual += x, x = layernorm(residual) * w + b (in place)
void llmd_layer_norm(void* out, int64_t out_stride, void* x, int64_t x_stride, void* residual, int64_t res_stride,
                     const void* w, const void* b, int rows, int d, float eps, hipStream_t st) {
  if (rows == 0) return;
  if (residual)
    launch_ln<true>(nullptr, 0, (uint16_t*)x, x_stride, (uint16_t*)residual, res_stride, (const uint16_t*)w,
                    (const uint16_t*)b, rows, d, eps, st);
  else
    launch_ln<false>((uint16_t*)out, out_stride, (uint16_t*)x, x_stride, nullptr, 0, (const uint16_t*)w,
                     (const uint16_t*)b, rows, d, eps, st);
}

// q, scale = fp8_per_row(rmsnorm(x [+ residual]) * w); residual updated in place when given
void llmd_rms_norm_quant(void* q, int64_t q_stride, float* scale, const void* x, int64_t x_stride, void* residual,
                         int64_t res_stride, const void* w, int rows, int d, float eps, hipStream_t st) {
  if (rows == 0) return;
  if (residual)
    launch_q<true>((uint8_t*)q, q_stride, scale, (const uint16_t*)x, x_stride, (uint16_t*)residual, res_stride,
                   (const uint16_t*)w, rows, d, eps, st);
  else
    launch_q<false>((uint8_t*)q, q_stride, scale, (const uint16_t*)x, x_stride, nullptr, 0, (const uint16_t*)w,
                    rows, d, eps, st);
}

// out[rows, d] = x * rsqrt(mean(x^2) + eps) * w
void llmd_rms_norm(void* out, int64_t out_stride, const void* x, int64_t x_stride,
                   const void* w, int rows, int d, float eps, hipStream_t st) {
  launch<false>((uint16_t*)out, out_stride, (uint16_t*)x, x_stride, nullptr, 0,
                (const uint16_t*)w, rows, d, eps, st);
}
// residual += x ; x = rmsnorm(residual) * w   (both in place)
void llmd_fused_add_rms_norm(void* x, int64_t x_stride, void* residual, int64_t res_stride,
                             const void* w, int rows, int d, float eps, hipStream_t st) {
  launch<true>(nullptr, 0, (uint16_t*)x, x_stride, (uint16_t*)residual, res_stride,
               (const uint16_t*)w, rows, d, eps, st);
}
}
