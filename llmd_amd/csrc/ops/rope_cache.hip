// Fused rotary embedding + paged KV-cache write (vLLM
// `rotary_embedding` + `reshape_and_cache` fused into one pass).
//
// Input is the raw output of the fused QKV projection, qkv[T, (Hq+2Hkv)*D].
//   * Q heads are rotated in place (the attention kernels read Q through a row stride).
//   * K heads are rotated and scattered into the paged cache at slot_mapping[t].
//   * V heads are copied into the paged cache.
// Paged cache layout (per layer view; see llmd_amd/engine/kv_cache.py):
//   element (block b, kv head h, row r, dim d) at  b*block_stride + h*bs*D + r*D + d
// with the K and V planes given as separate base pointers. A whole block of one
// layer is therefore one contiguous [Hkv, bs, D] slab, which is the unit moved by
// KV transfer (kvx) and offload.
// cos_sin[pos, 0:R/2] = cos, cos_sin[pos, R/2:R] = sin, f32, R = rotary dim.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

// NEOX = rotate_half pairing (d, d + R/2); otherwise GPT-J interleaved pairs (2i, 2i+1).
// F8: the cache is e4m3fn; K/V are multiplied by kinv/vinv (1/k_scale, 1/v_scale)
// and saturated on the way in (SURVEY K06 "quantize K/V", K16).
// One token row: `src` is the projection output row (global, or an LDS copy), rotated Q goes to
// `row` (the qkv buffer row the attention reads), rotated K and V to the cache. NTH threads.
template <bool NEOX, bool F8, int NTH>
__device__ __forceinline__ void rope_row(const uint16_t* src, uint16_t* row, int t,
                                         const int64_t* __restrict__ positions, const float* __restrict__ cos_sin,
                                         int rot, int Hq, int Hkv, int D, const int64_t* __restrict__ slots,
                                         void* __restrict__ kc, void* __restrict__ vc, int64_t block_stride, int bs,
                                         float kinv, float vinv) {
  const int64_t pos = positions[t];
  const float* cs = cos_sin + pos * rot;
  const int64_t slot = slots ? slots[t] : -1;
  LLMD_DCHECK(slot >= -1);  // -1 = padded row (graph buckets), else a cache slot
  int64_t cache_off = -1;
  if (slot >= 0) {
    const int64_t blk = slot / bs, r = slot % bs;
    cache_off = blk * block_stride + r * D;
  }
  const int half = rot / 2;
  // --- rotation work: (Hq + Hkv) heads x (rot/16) items of 8 pairs
  const int items_per_head = rot / 16;
  const int n_rot = (Hq + Hkv) * items_per_head;
  for (int it = threadIdx.x; it < n_rot; it += NTH) {
    const int h = it / items_per_head, c = it % items_per_head;
    const uint16_t* hp = src + h * D;
    float a[8], b[8], co[8], si[8];
    int ia, ib;  // element offsets of the two 8-wide operands
    if (NEOX) {
      ia = c * 8;
      ib = half + c * 8;
      u32x4_t va = *reinterpret_cast<const u32x4_t*>(hp + ia);
      u32x4_t vb = *reinterpret_cast<const u32x4_t*>(hp + ib);
      unpack8(va, a);
      unpack8(vb, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        co[j] = cs[c * 8 + j];
        si[j] = cs[half + c * 8 + j];
      }
    } else {
      // 16 consecutive elements = 8 interleaved pairs
      ia = c * 16;
      ib = c * 16 + 8;
      u32x4_t va = *reinterpret_cast<const u32x4_t*>(hp + ia);
      u32x4_t vb = *reinterpret_cast<const u32x4_t*>(hp + ib);
      float e[16];
      unpack8(va, e);
      unpack8(vb, e + 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = e[2 * j];
        b[j] = e[2 * j + 1];
        co[j] = cs[c * 8 + j];
        si[j] = cs[half + c * 8 + j];
      }
    }
    float oa[8], ob[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      oa[j] = a[j] * co[j] - b[j] * si[j];
      ob[j] = b[j] * co[j] + a[j] * si[j];
    }
    u32x4_t pa, pb;
    if (NEOX) {
      pa = pack8(oa);
      pb = pack8(ob);
    } else {
      float e[16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        e[2 * j] = oa[j];
        e[2 * j + 1] = ob[j];
      }
      pa = pack8(e);
      pb = pack8(e + 8);
    }
    if (h < Hq) {
      *reinterpret_cast<u32x4_t*>(row + h * D + ia) = pa;
      *reinterpret_cast<u32x4_t*>(row + h * D + ib) = pb;
    } else if (cache_off >= 0) {
      const int64_t dst = cache_off + (int64_t)(h - Hq) * bs * D;
      store8_from_bf16<F8>(kc, dst + ia, pa, kinv);
      store8_from_bf16<F8>(kc, dst + ib, pb, kinv);
    }
  }
  if (cache_off < 0) return;
  // --- K pass-through dims beyond the rotary dim, and V copy
  const int cpr = D / 8;             // 16-B chunks per head
  const int kpass = (D - rot) / 8;   // un-rotated K chunks per head
  const int n_copy = Hkv * (kpass + cpr);
  for (int it = threadIdx.x; it < n_copy; it += NTH) {
    const int per = kpass + cpr;
    const int h = it / per, c = it % per;
    if (c < kpass) {
      const int e = rot + c * 8;
      u32x4_t v = *reinterpret_cast<const u32x4_t*>(src + (Hq + h) * D + e);
      store8_from_bf16<F8>(kc, cache_off + (int64_t)h * bs * D + e, v, kinv);
    } else {
      const int e = (c - kpass) * 8;
      u32x4_t v = *reinterpret_cast<const u32x4_t*>(src + (Hq + Hkv + h) * D + e);
      store8_from_bf16<F8>(vc, cache_off + (int64_t)h * bs * D + e, v, vinv);
    }
  }
}

template <bool NEOX, bool F8>
__global__ __launch_bounds__(NT) void rope_cache_kernel(
    uint16_t* __restrict__ qkv, int64_t qkv_stride, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, int rot, int Hq, int Hkv, int D,
    const int64_t* __restrict__ slots, void* __restrict__ kc, void* __restrict__ vc,
    int64_t block_stride, int bs, float kinv, float vinv) {
  const int t = blockIdx.x;
  uint16_t* row = qkv + (int64_t)t * qkv_stride;
  rope_row<NEOX, F8, NT>(row, row, t, positions, cos_sin, rot, Hq, Hkv, D, slots, kc, vc, block_stride, bs, kinv,
                         vinv);
}

// The decode step's QKV projection split-K partials (fp32 [nsplit][T][W], csrc/ops/mgemm.hip) summed
// and rounded to bf16 exactly as mgemm_reduce_kernel does, staged in LDS (and stored to the qkv row),
// then RoPE + the paged cache write from the LDS copy: one launch instead of reduce + rope_cache,
// bit-identical to them. 1024 threads per token row (the partials stream with enough loads in flight).
constexpr int RNT = 1024;
constexpr int RMAXW = 24576;  // row width (elements) the 48 KB LDS copy holds

template <bool NEOX, bool F8>
__global__ __launch_bounds__(RNT) void reduce_rope_cache_kernel(
    const float* __restrict__ part, int nsplit, int T, int W, uint16_t* __restrict__ qkv, int64_t qkv_stride,
    const int64_t* __restrict__ positions, const float* __restrict__ cos_sin, int rot, int Hq, int Hkv, int D,
    const int64_t* __restrict__ slots, void* __restrict__ kc, void* __restrict__ vc, int64_t block_stride, int bs,
    float kinv, float vinv) {
  __shared__ __attribute__((aligned(16))) uint16_t lrow[RMAXW];
  const int t = blockIdx.x;
  const int64_t total = (int64_t)T * W;
  uint16_t* row = qkv + (int64_t)t * qkv_stride;
  for (int c = threadIdx.x; c < W / 8; c += RNT) {
    const float* p = part + (int64_t)t * W + c * 8;
    f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(p), s1 = *reinterpret_cast<const f32x4_t*>(p + 4);
    for (int k = 1; k < nsplit; ++k) {
      s0 += *reinterpret_cast<const f32x4_t*>(p + (int64_t)k * total);
      s1 += *reinterpret_cast<const f32x4_t*>(p + (int64_t)k * total + 4);
    }
    const float y[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    const u32x4_t v = pack8(y);
    *reinterpret_cast<u32x4_t*>(lrow + c * 8) = v;
    *reinterpret_cast<u32x4_t*>(row + c * 8) = v;  // the un-rotated projection, as the two-kernel path leaves K / V
  }
  __syncthreads();
  rope_row<NEOX, F8, RNT>(lrow, row, t, positions, cos_sin, rot, Hq, Hkv, D, slots, kc, vc, block_stride, bs, kinv,
                          vinv);
}

}  // namespace

extern "C" int llmd_reduce_rope_cache(const float* part, int nsplit, int W, void* qkv, int64_t qkv_stride,
                                      const int64_t* positions, const float* cos_sin, int rot, int Hq, int Hkv,
                                      int D, const int64_t* slots, void* kc, void* vc, int64_t block_stride, int bs,
                                      int T, int neox, int fp8, float kinv, float vinv, hipStream_t st) {
  if (T == 0) return 0;
  if (W % 8 || W > RMAXW || W < (Hq + 2 * Hkv) * D || qkv_stride % 8 || nsplit < 1) return -1;
  dim3 g(T), b(RNT);
#define LAUNCH(NX, F8)                                                                                          \
  hipLaunchKernelGGL((reduce_rope_cache_kernel<NX, F8>), g, b, 0, st, part, nsplit, T, W, (uint16_t*)qkv,       \
                     qkv_stride, positions, cos_sin, rot, Hq, Hkv, D, slots, kc, vc, block_stride, bs, kinv, vinv)
  if (neox) {
    if (fp8) LAUNCH(true, true); else LAUNCH(true, false);
  } else {
    if (fp8) LAUNCH(false, true); else LAUNCH(false, false);
  }
#undef LAUNCH
  return (int)hipGetLastError();
}

extern "C" void llmd_rope_cache(void* qkv, int64_t qkv_stride, const int64_t* positions,
                                const float* cos_sin, int rot, int Hq, int Hkv, int D,
                                const int64_t* slots, void* kc, void* vc, int64_t block_stride,
                                int bs, int T, int neox, int fp8, float kinv, float vinv, hipStream_t st) {
  if (T == 0) return;
  dim3 g(T), b(NT);
#define LAUNCH(NX, F8)                                                                                \
  hipLaunchKernelGGL((rope_cache_kernel<NX, F8>), g, b, 0, st, (uint16_t*)qkv, qkv_stride, positions, \
                     cos_sin, rot, Hq, Hkv, D, slots, kc, vc, block_stride, bs, kinv, vinv)
  if (neox) {
    if (fp8) LAUNCH(true, true); else LAUNCH(true, false);
  } else {
    if (fp8) LAUNCH(false, true); else LAUNCH(false, false);
  }
#undef LAUNCH
}
