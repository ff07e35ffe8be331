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
template <bool NEOX, bool F8>
__global__ __launch_bounds__(NT) void rope_cache_kernel(
    uint16_t* __restrict__ qkv, int64_t qkv_stride, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, int rot, int Hq, int Hkv, int D,
    const int64_t* __restrict__ slots, void* __restrict__ kc, void* __restrict__ vc,
    int64_t block_stride, int bs, float kinv, float vinv) {
  const int t = blockIdx.x;
  const int64_t pos = positions[t];
  const float* cs = cos_sin + pos * rot;
  uint16_t* row = qkv + (int64_t)t * qkv_stride;
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
  for (int it = threadIdx.x; it < n_rot; it += NT) {
    const int h = it / items_per_head, c = it % items_per_head;
    uint16_t* hp = row + h * D;
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
      *reinterpret_cast<u32x4_t*>(hp + ia) = pa;
      *reinterpret_cast<u32x4_t*>(hp + ib) = pb;
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
  for (int it = threadIdx.x; it < n_copy; it += NT) {
    const int per = kpass + cpr;
    const int h = it / per, c = it % per;
    if (c < kpass) {
      const int e = rot + c * 8;
      u32x4_t v = *reinterpret_cast<const u32x4_t*>(row + (Hq + h) * D + e);
      store8_from_bf16<F8>(kc, cache_off + (int64_t)h * bs * D + e, v, kinv);
    } else {
      const int e = (c - kpass) * 8;
      u32x4_t v = *reinterpret_cast<const u32x4_t*>(row + (Hq + Hkv + h) * D + e);
      store8_from_bf16<F8>(vc, cache_off + (int64_t)h * bs * D + e, v, vinv);
    }
  }
}

}  // namespace

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
