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

}  // namespace

extern "C" {
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
