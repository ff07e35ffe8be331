// Paged decode attention, GQA, split-K ("flash-decoding") on MFMA.
//
// Grid (split, kv_head x head_group, seq); 256 threads = 4 independent waves.
// Each wave walks 64-key tiles of its split (tile w, w+4, ...) with its own
// online-softmax state, and the four waves are merged through LDS at the end.
//
// Per 64-key tile and wave:
//   S^T[key][head] = K[key][:] . Q[head][:]   4 x D/32 mfma_f32_16x16x32_bf16
//     A = K rows straight from HBM (16 B per lane, 64 contiguous bytes per row
//         per instruction), B = Q fragments held in registers.
//     Keys sit on the MFMA M axis, so the softmax probabilities come out
//     lane-local in exactly the layout of the next product's A operand.
//   O[head][dim] += P[head][key] . V[key][dim]  2 x D/16 MFMAs
//     V is staged through a per-wave XOR-swizzled LDS image and consumed with
//     ds_read_b64_tr_b16 (hardware transpose) - conflict-free on 2^n rows.
// The key<->MFMA-row permutation `rowoff` is chosen so a half-wave's two
// transposed-read blocks sit 8 rows apart (bank-conflict free) while P stays
// lane-local.
//
// Query heads of one KV head ride the MFMA N axis (16 wide): G <= 16 per pass,
// larger groups are split into head groups (grid.y = Hkv * NG).
// Sliding window (gpt-oss) and attention sinks are supported; the sink only
// enters the final normaliser.
// Partial results (unnormalised O, running max M and sum L in log2 units) go to
// a workspace when nsplit > 1 and are merged by `decode_reduce_kernel`.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;
constexpr float NEG_INF = -__builtin_huge_valf();

__device__ __forceinline__ int rowoff(int g) { return 4 * (g >> 1) + 8 * (g & 1); }

// byte offset of 16-B chunk `ch` of LDS row `row` in a [64][D] bf16 image
template <int D>
__device__ __forceinline__ int vimg_off(int row, int ch) {
  if constexpr (D == 128) {
    const int sw = ((row & 3) << 2) | ((row >> 2) & 3);
    return row * 256 + 16 * (ch ^ sw);
  } else {  // D == 64: 128-B rows, two rows per 256-B bank row
    const int sw = 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
    return row * 128 + 16 * (ch ^ sw);
  }
}

// Raw cache registers: bf16 keeps 16 B per 8 elements, fp8 (e4m3fn) 8 B. fp8
// values stay packed while their loads are in flight and are widened to bf16
// (exact) right before the MFMA / LDS staging, so the prefetch distance is
// unchanged and the K/V bytes read from HBM halve. k_scale is folded into the
// softmax scale on the host, v_scale into the output (`vscale`).
template <bool F8>
struct CacheReg {
  using T = u32x4_t;
};
template <>
struct CacheReg<true> {
  using T = u32x2_t;
};
template <bool F8>
__device__ __forceinline__ typename CacheReg<F8>::T ld_cache(const void* base, int64_t off) {
  if constexpr (F8)
    return *reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(base) + off);
  else
    return *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(base) + off);
}
template <bool F8>
__device__ __forceinline__ u32x4_t widen(const typename CacheReg<F8>::T v) {
  if constexpr (F8)
    return fp8x8_to_bf16x8(v);
  else
    return v;
}

template <int D, bool F8>
__global__ __launch_bounds__(NT, 2) void paged_decode_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const void* __restrict__ kc,
    const void* __restrict__ vc, int64_t block_stride, int bs,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    int Hq, int Hkv, int G, int NG, float scale_log2, int window,
    const float* __restrict__ sinks, int split_size, int nsplit, uint16_t* __restrict__ out,
    int64_t out_stride, float* __restrict__ part_o, float* __restrict__ part_ml, float vscale) {
  using CR = typename CacheReg<F8>::T;
  constexpr int KS = D / 32;   // k-steps of the QK^T product
  constexpr int NB = D / 16;   // 16-wide dim blocks of the PV product
  constexpr int CPR = D / 8;   // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per V load instruction
  constexpr int VLD = CPR;     // V load instructions per tile per lane
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int sp = blockIdx.x;
  const int kvh = blockIdx.y / NG, gi = blockIdx.y % NG;
  const int b = blockIdx.z;
  const int L = seq_lens[b];
  LLMD_DCHECK(L >= 0 && L <= bt_stride * bs);  // the block table covers the sequence
  const int start = window > 0 ? max(0, L - window) : 0;
  const int s0 = start + sp * split_size;
  if (s0 >= L) return;
  const int s1 = min(s0 + split_size, L);
  const int h0 = kvh * G + gi * 16;
  const int nh = min(16, G - gi * 16);

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, c16 = lane & 15;
  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);  // block size is a power of two (checked on the host)

  // ---- Q fragments (B operand of S^T = K Q^T)
  bf16x8_t qf[KS];
  {
    const uint16_t* qr = q + (int64_t)b * q_stride + (int64_t)(h0 + c16) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (c16 < nh) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      qf[s] = __builtin_bit_cast(bf16x8_t, v);
    }
  }

  float m = NEG_INF, lsum = 0.f;
  f32x4_t o[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  char* vimg = smem + w * (64 * D * 2);
  const int ntile = (s1 - s0 + 63) >> 6;

  // K of tile t is loaded one iteration ahead (issued right after the
  // previous tile's S product retires its registers), V of tile t is issued
  // at the top of the iteration: its latency hides behind S + softmax, K's
  // behind the whole previous PV. Register footprint stays one K + one V set.
  CR kf[4][KS];
  auto load_k = [&](int tt) {
    const int tts = s0 + 64 * tt;
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      int key = tts + 16 * b4 + rowoff(c16 >> 2) + (c16 & 3);
      key = key < s1 ? key : s0;
      const int phys = bt[key >> lbs];
      LLMD_DCHECK(phys >= 0);
      const int64_t kr = (int64_t)phys * block_stride + head_off + (int64_t)(key & (bs - 1)) * D;
#pragma unroll
      for (int s = 0; s < KS; ++s) kf[b4][s] = ld_cache<F8>(kc, kr + (4 * s + g) * 8);
    }
  };
  if (w < ntile) load_k(w);

  for (int t = w; t < ntile; t += 4) {
    const int ts = s0 + 64 * t;
    CR vr[VLD];
#pragma unroll
    for (int i = 0; i < VLD; ++i) {
      const int row = i * RPI + lane / CPR;
      int key = ts + row;
      key = key < s1 ? key : s0;
      const int phys = bt[key >> lbs];
      const int64_t vp = (int64_t)phys * block_stride + head_off + (int64_t)(key & (bs - 1)) * D;
      vr[i] = ld_cache<F8>(vc, vp + (lane % CPR) * 8);
    }
    // ---- S^T = K Q^T
    f32x4_t sc[4];
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, widen<F8>(kf[b4][s])),
                                                      qf[s], acc, 0, 0, 0);
      sc[b4] = acc;
    }
    if (t + 4 < ntile) load_k(t + 4);
    // ---- online softmax (log2 domain); element i of group g is key ts+16*b4+rowoff(g)+i
    float mx = NEG_INF;
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = ts + 16 * b4 + rowoff(g) + i;
        float v = sc[b4][i] * scale_log2;
        v = key < s1 ? v : NEG_INF;
        sc[b4][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = exp2f(m - mnew);
    float ps = 0.f;
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(sc[b4][i] - mnew);
        sc[b4][i] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    lsum = lsum * alpha + ps;
    m = mnew;
    // rescale O rows (row = head 4g+i; that head's alpha lives in lane 4g+i)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
      for (int n = 0; n < NB; ++n) o[n][i] *= a;
    }
    // ---- stage V into this wave's swizzled LDS image
#pragma unroll
    for (int i = 0; i < VLD; ++i) {
      const int row = i * RPI + lane / CPR;
      *reinterpret_cast<u32x4_t*>(vimg + vimg_off<D>(row, lane % CPR)) = widen<F8>(vr[i]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- O += P V
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      bf16x8_t pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = (__bf16)sc[2 * t2][j];
        pa[4 + j] = (__bf16)sc[2 * t2 + 1][j];
      }
      const int qq = c16 >> 2, pp = c16 & 3;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int r0 = 32 * t2 + rowoff(g) + qq;
        const int ch = 2 * n + (pp >> 1);
        const int a0 = vimg_off<D>(r0, ch) + 8 * (pp & 1);
        const int a1 = vimg_off<D>(r0 + 16, ch) + 8 * (pp & 1);
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(vimg + a0));
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(vimg + a1));
        s16x8_t vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8_t, vb), o[n],
                                                       0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // ---- merge the 4 waves: m/l per head, O rows
  __syncthreads();
  float* ml = reinterpret_cast<float*>(smem);                 // [4 waves][16 heads][2]
  float* ob = reinterpret_cast<float*>(smem + 4 * 16 * 2 * 4);  // [4][16][D]
  if (g == 0) {
    ml[(w * 16 + c16) * 2 + 0] = m;
    ml[(w * 16 + c16) * 2 + 1] = lsum;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = 4 * g + i;
    float M = NEG_INF;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, ml[(ww * 16 + h) * 2]);
    const float mine = ml[(w * 16 + h) * 2];
    const float f = (mine == NEG_INF) ? 0.f : exp2f(mine - M);
#pragma unroll
    for (int n = 0; n < NB; ++n) ob[(w * 16 + h) * D + 16 * n + c16] = o[n][i] * f;
  }
  __syncthreads();
  // 16 heads x D outputs over 256 threads
  for (int e = threadIdx.x; e < 16 * D; e += NT) {
    const int h = e / D, d = e % D;
    if (h >= nh) continue;
    float M = NEG_INF;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, ml[(ww * 16 + h) * 2]);
    float Ls = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float mw = ml[(ww * 16 + h) * 2];
      const float f = (mw == NEG_INF) ? 0.f : exp2f(mw - M);
      Ls += f * ml[(ww * 16 + h) * 2 + 1];
      acc += ob[(ww * 16 + h) * D + d];
    }
    acc *= vscale;
    const int hq = h0 + h;
    if (nsplit == 1) {
      float den = Ls;
      if (sinks) den += exp2f(sinks[hq] * 1.4426950408889634f - M);
      out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(acc / den);
    } else {
      const int64_t pi = ((int64_t)b * Hq + hq) * nsplit + sp;
      part_o[pi * D + d] = acc;
      if (d == 0) {
        part_ml[pi * 2] = M;
        part_ml[pi * 2 + 1] = Ls;
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(64) void decode_reduce_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_ml,
    const int* __restrict__ seq_lens, int Hq, int nsplit, int split_size, int window,
    const float* __restrict__ sinks, uint16_t* __restrict__ out, int64_t out_stride) {
  const int hq = blockIdx.x, b = blockIdx.y;
  const int L = seq_lens[b];
  const int start = window > 0 ? max(0, L - window) : 0;
  const int nact = min(nsplit, (L - start + split_size - 1) / split_size);
  const int64_t base = ((int64_t)b * Hq + hq) * nsplit;
  float M = NEG_INF;
  for (int s = 0; s < nact; ++s) M = fmaxf(M, part_ml[(base + s) * 2]);
  float den = 0.f;
  for (int s = 0; s < nact; ++s) den += exp2f(part_ml[(base + s) * 2] - M) * part_ml[(base + s) * 2 + 1];
  if (sinks) den += exp2f(sinks[hq] * 1.4426950408889634f - M);
  const float inv = 1.f / den;
  for (int d = threadIdx.x; d < D; d += 64) {
    float acc = 0.f;
    for (int s = 0; s < nact; ++s) acc += exp2f(part_ml[(base + s) * 2] - M) * part_o[(base + s) * D + d];
    out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(acc * inv);
  }
}

}  // namespace

extern "C" int llmd_paged_decode(const void* q, int64_t q_stride, const void* kc, const void* vc,
                                 int64_t block_stride, int bs, const int* block_tables,
                                 int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int D,
                                 float scale, int window, const float* sinks, int split_size,
                                 int nsplit, void* out, int64_t out_stride, float* part_o,
                                 float* part_ml, int fp8, float k_scale, float v_scale, hipStream_t st) {
  if (B == 0) return 0;
  const int G = Hq / Hkv;
  const int NG = (G + 15) / 16;
  const float scale_log2 = scale * k_scale * 1.4426950408889634f;
  dim3 grid(nsplit, Hkv * NG, B), blk(NT);
  const size_t lds = (size_t)4 * 64 * D * 2;
#define LAUNCH(DD, F8)                                                                                    \
  do {                                                                                                    \
    hipLaunchKernelGGL((paged_decode_kernel<DD, F8>), grid, blk, lds, st, (const uint16_t*)q, q_stride, kc, \
                       vc, block_stride, bs, block_tables, bt_stride, seq_lens, Hq, Hkv, G, NG, scale_log2, \
                       window, sinks, split_size, nsplit, (uint16_t*)out, out_stride, part_o, part_ml,     \
                       v_scale);                                                                          \
    if (nsplit > 1)                                                                                       \
      hipLaunchKernelGGL(decode_reduce_kernel<DD>, dim3(Hq, B), dim3(64), 0, st, part_o, part_ml, seq_lens, \
                         Hq, nsplit, split_size, window, sinks, (uint16_t*)out, out_stride);                \
  } while (0)
  if (D == 128) {
    if (fp8) LAUNCH(128, true); else LAUNCH(128, false);
  } else if (D == 64) {
    if (fp8) LAUNCH(64, true); else LAUNCH(64, false);
  } else {
    return -1;
  }
#undef LAUNCH
  return 0;
}
