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
// NTL: non-temporal (nt) loads - the K/V of a decode step is read once, and a
// layer's cache (1.3 GB at 64 x 5000 tokens for 70B) never fits the 256 MB MALL
template <bool F8, bool NTL = false>
__device__ __forceinline__ typename CacheReg<F8>::T ld_cache(const void* base, int64_t off) {
  if constexpr (F8) {
    const u32x2_t* p = reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(base) + off);
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    return *p;
  } else {
    const u32x4_t* p = reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(base) + off);
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    return *p;
  }
}
template <bool F8>
__device__ __forceinline__ u32x4_t widen(const typename CacheReg<F8>::T v) {
  if constexpr (F8)
    return fp8x8_to_bf16x8(v);
  else
    return v;
}

// ---- the 64-key tile loop shared by the per-sequence and the shared-prefix
// kernels. NP passes of 16 query columns ride the same K registers and the same
// staged V image: a shared prefix is read from HBM once for all of them.
template <int D, bool F8, int NP>
struct TileState {
  bf16x8_t qf[NP][D / 32];
  f32x4_t o[NP][D / 16];
  float m[NP], lsum[NP];
};

template <int D, bool F8, int NP, bool NTL = false>
__device__ __forceinline__ void attend_tiles(TileState<D, F8, NP>& st, const void* __restrict__ kc,
                                             const void* __restrict__ vc, int64_t block_stride, int bs,
                                             const int* __restrict__ bt, int64_t head_off, int s0, int s1,
                                             float scale_log2, char* vimg, int w, int lane) {
  using CR = typename CacheReg<F8>::T;
  constexpr int KS = D / 32;   // k-steps of the QK^T product
  constexpr int NB = D / 16;   // 16-wide dim blocks of the PV product
  constexpr int CPR = D / 8;   // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per V load instruction
  constexpr int VLD = CPR;     // V load instructions per tile per lane
  const int g = lane >> 4, c16 = lane & 15;
  const int lbs = __builtin_ctz(bs);  // block size is a power of two (checked on the host)
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
      for (int s = 0; s < KS; ++s) kf[b4][s] = ld_cache<F8, NTL>(kc, kr + (4 * s + g) * 8);
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
      vr[i] = ld_cache<F8, NTL>(vc, vp + (lane % CPR) * 8);
    }
    // ---- S^T = K Q^T for every pass
    f32x4_t sc[NP][4];
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, widen<F8>(kf[b4][s])),
                                                        st.qf[p][s], acc, 0, 0, 0);
        sc[p][b4] = acc;
      }
    if (t + 4 < ntile) load_k(t + 4);
    // ---- online softmax (log2 domain); element i of group g is key ts+16*b4+rowoff(g)+i
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float mx = NEG_INF;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = ts + 16 * b4 + rowoff(g) + i;
          float v = sc[p][b4][i] * scale_log2;
          v = key < s1 ? v : NEG_INF;
          sc[p][b4][i] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(st.m[p], mx);
      const float alpha = exp2f(st.m[p] - mnew);
      float ps = 0.f;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = exp2f(sc[p][b4][i] - mnew);
          sc[p][b4][i] = pv;
          ps += pv;
        }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      st.lsum[p] = st.lsum[p] * alpha + ps;
      st.m[p] = mnew;
      // rescale O rows (row = column 4g+i; that column's alpha lives in lane 4g+i)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
        for (int n = 0; n < NB; ++n) st.o[p][n][i] *= a;
      }
    }
    // ---- stage V into this wave's swizzled LDS image
#pragma unroll
    for (int i = 0; i < VLD; ++i) {
      const int row = i * RPI + lane / CPR;
      *reinterpret_cast<u32x4_t*>(vimg + vimg_off<D>(row, lane % CPR)) = widen<F8>(vr[i]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- O += P V (one transposed V fragment read serves every pass)
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      bf16x8_t pa[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[p][j] = (__bf16)sc[p][2 * t2][j];
          pa[p][4 + j] = (__bf16)sc[p][2 * t2 + 1][j];
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
#pragma unroll
        for (int p = 0; p < NP; ++p)
          st.o[p][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[p], __builtin_bit_cast(bf16x8_t, vb),
                                                               st.o[p][n], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// ---- merge pass p of the 4 waves through LDS; emit(col, d, acc, M, Ls) per
// output element (16 columns x D over the 256 threads), acc unnormalised.
template <int D, bool F8, int NP, typename Emit>
__device__ __forceinline__ void merge_waves(const TileState<D, F8, NP>& st, int p, char* smem, int w,
                                            int lane, Emit emit) {
  constexpr int NB = D / 16;
  const int g = lane >> 4, c16 = lane & 15;
  __syncthreads();
  float* ml = reinterpret_cast<float*>(smem);                 // [4 waves][16 cols][2]
  float* ob = reinterpret_cast<float*>(smem + 4 * 16 * 2 * 4);  // [4][16][D]
  if (g == 0) {
    ml[(w * 16 + c16) * 2 + 0] = st.m[p];
    ml[(w * 16 + c16) * 2 + 1] = st.lsum[p];
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
    for (int n = 0; n < NB; ++n) ob[(w * 16 + h) * D + 16 * n + c16] = st.o[p][n][i] * f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * D; e += NT) {
    const int h = e / D, d = e % D;
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
    emit(h, d, acc, M, Ls);
  }
}

// One sequence's keys [start, L) (start = sliding-window start, or the end of
// its shared prefix `sstart[b]` when the shared-prefix kernel covers the rest).
// direct: one split and no shared prefix - normalise and write `out` here;
// otherwise partial slot `sp` of nslot per (seq, head).
template <int D, bool F8, bool NTL = false>
__global__ __launch_bounds__(NT, 2) void paged_decode_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const void* __restrict__ kc,
    const void* __restrict__ vc, int64_t block_stride, int bs,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    const int* __restrict__ sstart, int Hq, int Hkv, int G, int NG, float scale_log2, int window,
    const float* __restrict__ sinks, int split_size, const int* __restrict__ split_dev, int nslot, int direct,
    uint16_t* __restrict__ out, int64_t out_stride, float* __restrict__ part_o, float* __restrict__ part_ml,
    float vscale) {
  constexpr int KS = D / 32;
  constexpr int NB = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int sp = blockIdx.x;
  const int kvh = blockIdx.y / NG, gi = blockIdx.y % NG;
  const int b = blockIdx.z;
  const int L = seq_lens[b];
  LLMD_DCHECK(L >= 0 && L <= bt_stride * bs);  // the block table covers the sequence
  int start = window > 0 ? max(0, L - window) : 0;
  if (sstart) start = max(start, sstart[b]);
  if (split_dev) split_size = *split_dev;  // hipGraph replay: keys per split sized to this step's contexts
  const int s0 = start + sp * split_size;
  if (s0 >= L) return;
  const int s1 = min(s0 + split_size, L);
  const int h0 = kvh * G + gi * 16;
  const int nh = min(16, G - gi * 16);

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, c16 = lane & 15;
  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;

  TileState<D, F8, 1> st;
  {  // Q fragments (B operand of S^T = K Q^T)
    const uint16_t* qr = q + (int64_t)b * q_stride + (int64_t)(h0 + c16) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (c16 < nh) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      st.qf[0][s] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  st.m[0] = NEG_INF;
  st.lsum[0] = 0.f;
#pragma unroll
  for (int n = 0; n < NB; ++n) st.o[0][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  attend_tiles<D, F8, 1, NTL>(st, kc, vc, block_stride, bs, bt, head_off, s0, s1, scale_log2,
                         smem + w * (64 * D * 2), w, lane);

  merge_waves<D, F8, 1>(st, 0, smem, w, lane, [&](int h, int d, float acc, float M, float Ls) {
    if (h >= nh) return;
    acc *= vscale;
    const int hq = h0 + h;
    if (direct) {
      float den = Ls;
      if (sinks) den += exp2f(sinks[hq] * 1.4426950408889634f - M);
      out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(acc / den);
    } else {
      const int64_t pi = ((int64_t)b * Hq + hq) * nslot + sp;
      part_o[pi * D + d] = acc;
      if (d == 0) {
        part_ml[pi * 2] = M;
        part_ml[pi * 2 + 1] = Ls;
      }
    }
  });
}

// Shared-prefix ("cascade") decode: one work unit = up to 16*NP/G sequences
// whose first `hi` keys are the same physical blocks, and a key range [lo, hi)
// of that prefix. Every member's G query heads take 16*NP MFMA columns, so the
// prefix K/V is read once for all of them; partials go to slot pslot0 + `slot`
// of each member (after its own nsplit suffix slots) and are merged with its
// suffix by decode_reduce_kernel.
// work: int32 [nwork][5] = {first member (index into `members`), members, lo, hi, slot};
// units with 0 members are padding (fixed grid under hipGraph capture).
template <int D, bool F8, int NP>
__global__ __launch_bounds__(NT, NP == 1 ? 2 : 1) void shared_prefix_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const void* __restrict__ kc,
    const void* __restrict__ vc, int64_t block_stride, int bs, const int* __restrict__ block_tables,
    int bt_stride, const int* __restrict__ members, const int* __restrict__ work, int Hq, int G,
    float scale_log2, int nslot, int pslot0, float* __restrict__ part_o, float* __restrict__ part_ml,
    float vscale) {
  constexpr int KS = D / 32;
  constexpr int NB = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int kvh = blockIdx.x;
  const int* wk = work + blockIdx.y * 5;
  const int m0 = wk[0], nm = wk[1], s0 = wk[2], s1 = wk[3], slot = wk[4];
  if (nm <= 0 || s0 >= s1) return;
  const int spp = 16 / G;  // members per 16-column pass (host: 16 % G == 0, nm <= spp*NP)
  LLMD_DCHECK(nm <= spp * NP && s1 <= bt_stride * bs);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, c16 = lane & 15;
  const int* bt = block_tables + (int64_t)members[m0] * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;

  TileState<D, F8, NP> st;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int mi = p * spp + c16 / G;
    const bool valid = mi < nm;
    const int b = valid ? members[m0 + mi] : 0;
    const uint16_t* qr = q + (int64_t)b * q_stride + (int64_t)(kvh * G + c16 % G) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (valid) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      st.qf[p][s] = __builtin_bit_cast(bf16x8_t, v);
    }
    st.m[p] = NEG_INF;
    st.lsum[p] = 0.f;
#pragma unroll
    for (int n = 0; n < NB; ++n) st.o[p][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  attend_tiles<D, F8, NP>(st, kc, vc, block_stride, bs, bt, head_off, s0, s1, scale_log2,
                          smem + w * (64 * D * 2), w, lane);

#pragma unroll
  for (int p = 0; p < NP; ++p)
    merge_waves<D, F8, NP>(st, p, smem, w, lane, [&](int c, int d, float acc, float M, float Ls) {
      const int mi = p * spp + c / G;
      if (mi >= nm || c >= spp * G) return;
      const int b = members[m0 + mi];
      const int hq = kvh * G + c % G;
      const int64_t pi = ((int64_t)b * Hq + hq) * nslot + pslot0 + slot;
      part_o[pi * D + d] = acc * vscale;
      if (d == 0) {
        part_ml[pi * 2] = M;
        part_ml[pi * 2 + 1] = Ls;
      }
    });
}

// ---- shared-prefix v2 (bf16 cache, D = 64/128, G = 4 or 8, block size >= 8
// keys): the prefix's 64-key K/V tiles move global -> LDS by DMA
// (global_load_lds_dwordx4, double-buffered, no VGPR staging) with
// attn_prefill.hip's prefill_v2 chunk swizzles applied on the source side, and
// all 4 waves read the same tiles. Each wave holds 32 query columns: G = 8 two
// heads x 16 members, G = 4 one head x 32 members, so one work unit serves up
// to 128/G members (all G heads) and reads its prefix range once.
template <int D>
__device__ __forceinline__ int sp_pk(int r) {
  if constexpr (D == 128) return ((r >> 1) & 7) | ((r & 1) << 3);
  else return (r & 2) | ((r >> 1) & 4);
}
template <int D>
__device__ __forceinline__ int sp_pv(int r) {
  if constexpr (D == 128) return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
  else return (r & 2) | ((r >> 1) & 4);
}

template <int D>
__global__ __launch_bounds__(NT, 2) void shared_prefix_v2_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int64_t block_stride, int bs, const int* __restrict__ block_tables,
    int bt_stride, const int* __restrict__ members, const int* __restrict__ work, int Hq, int G,
    float scale_log2, int nslot, int pslot0, float* __restrict__ part_o, float* __restrict__ part_ml,
    float vscale) {
  constexpr int KS = D / 32, NB = D / 16, RB = 2 * D;  // row bytes
  constexpr int IMG = 64 * RB;                          // one 64-key bf16 image
  constexpr int NI = 64 * (D / 8) / 64;                 // DMA wave-instructions per image (16 / 8)
  __shared__ __attribute__((aligned(1024))) char buf0[2 * IMG];  // K | V of even tiles
  __shared__ __attribute__((aligned(1024))) char buf1[2 * IMG];  // K | V of odd tiles
  const int kvh = blockIdx.x;
  const int* wk = work + blockIdx.y * 5;
  const int m0 = wk[0], nm = wk[1], lo = wk[2], hi = wk[3], slot = wk[4];
  if (nm <= 0 || lo >= hi) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const bool two_heads = G == 8;  // else G == 4 (host-checked)
  LLMD_DCHECK(nm <= (two_heads ? 16 : 32) && lo % 64 == 0 && hi <= bt_stride * bs);
  const int* bt = block_tables + (int64_t)members[m0] * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);

  // query column (block nb, column c) -> member index / head
  auto col_member = [&](int nb, int c) { return two_heads ? c : 16 * nb + c; };
  auto col_head = [&](int nb) { return kvh * G + (two_heads ? 2 * w + nb : w); };
  bf16x8_t qf[2][KS];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int mi = col_member(nb, c16);
    const bool valid = mi < nm;
    const int b = valid ? members[m0 + mi] : 0;
    const uint16_t* qr = q + (int64_t)b * q_stride + (int64_t)col_head(nb) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (valid) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      qf[nb][s] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  float m[2] = {NEG_INF, NEG_INF}, lsum[2] = {0.f, 0.f};
  f32x4_t o[2][NB];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int n = 0; n < NB; ++n) o[nb][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // DMA: NI K + NI V wave-instructions of 1 KB per tile; wave w issues j = w + 4i
  const int ws = __builtin_amdgcn_readfirstlane(w);
  uint32_t koff[NI / 4], voff[NI / 4];
#pragma unroll
  for (int i = 0; i < NI / 4; ++i) {
    const int u = 64 * (w + 4 * i) + lane;
    const int row = u / (D / 8), sl = u % (D / 8);
    koff[i] = (uint32_t)(row * RB + 16 * (sl ^ sp_pk<D>(row)));
    voff[i] = (uint32_t)(row * RB + 16 * (sl ^ sp_pv<D>(row)));
  }
  // one wave-instruction moves RPI consecutive rows, which sit in one cache
  // block (bs >= RPI): one scalar block-table lookup per instruction
  constexpr int RPI = 1024 / RB;
  auto issue = [&](char* base, int t) {
    const int ts = lo + 64 * t;
    const int rlim = hi - 1 - ts;
    if (rlim >= 63) {
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        const int r0 = RPI * (ws + 4 * i);
        const int key0 = ts + r0;
        LLMD_DCHECK(key0 < hi && bt[key0 >> lbs] >= 0);
        const int64_t tb = 2 * ((int64_t)bt[key0 >> lbs] * block_stride + head_off +
                                (int64_t)(key0 & (bs - 1)) * D) - (int64_t)r0 * RB;
        char* dst = base + 1024 * (ws + 4 * i);
        glds16(reinterpret_cast<const char*>(kc) + tb + koff[i], lds_addr(dst));  // asm DMA: counted lgkmcnt
        glds16(reinterpret_cast<const char*>(vc) + tb + voff[i], lds_addr(dst + IMG));
      }
    } else {  // last partial tile: rows past the prefix re-read key hi - 1 (finite; masked below)
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        const int u = 64 * (w + 4 * i) + lane;
        const int row = u / (D / 8), sl = u % (D / 8);
        const int key = ts + min(row, rlim);
        const int64_t ro = 2 * ((int64_t)bt[key >> lbs] * block_stride + head_off + (int64_t)(key & (bs - 1)) * D);
        char* dst = base + 1024 * (ws + 4 * i);
        glds16(reinterpret_cast<const char*>(kc) + ro + 16 * (sl ^ sp_pk<D>(row)), lds_addr(dst));
        glds16(reinterpret_cast<const char*>(vc) + ro + 16 * (sl ^ sp_pv<D>(row)), lds_addr(dst + IMG));
      }
    }
  };
  const int qq = c16 >> 2, pp = c16 & 3;
  const int srow = rowoff(c16 >> 2) + (c16 & 3), kp = sp_pk<D>(srow);
  int kofs[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) kofs[s] = srow * RB + 16 * ((4 * s + g) ^ kp);
  const int vrow = rowoff(g) + qq, vp = sp_pv<D>(vrow);
  int vofs[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) vofs[n] = IMG + vrow * RB + 16 * ((2 * n + (pp >> 1)) ^ vp) + 8 * (pp & 1);

  auto compute = [&](const char* img, int t) {
    const int ts = lo + 64 * t;
    f32x4_t sc[4][2];
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8_t ka = *reinterpret_cast<const bf16x8_t*>(img + kofs[s] + b4 * 16 * RB);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[0][s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[1][s], a1, 0, 0, 0);
      }
      sc[b4][0] = a0;
      sc[b4][1] = a1;
    }
    if (ts + 63 >= hi) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = ts + 16 * b4 + rowoff(g) + i;
            sc[b4][nb][i] = key < hi ? sc[b4][nb][i] : NEG_INF;
          }
    }
    // lazy rescale (attn_prefill.hip): only when a lane-local max exceeds m + 8
    float mt[2];
    bool grow = false;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float mx = NEG_INF;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[b4][nb][i]);
      mt[nb] = mx * scale_log2;
      grow = grow || (mt[nb] > m[nb] + 8.f);
    }
    if (__ballot(grow) != 0) {  // wave-uniform
      float alpha[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        float mx = fmaxf(mt[nb], __shfl_xor(mt[nb], 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[nb], mx);
        alpha[nb] = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m[nb] - mnew);
        lsum[nb] *= alpha[nb];
        m[nb] = mnew;
      }
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = __shfl(alpha[nb], 4 * g + i, 64);
#pragma unroll
          for (int n = 0; n < NB; ++n) o[nb][n][i] *= a;
        }
    }
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const float msub = (m[nb] == NEG_INF) ? 0.f : m[nb];
      float ps = 0.f;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[b4][nb][i], scale_log2, -msub));
          sc[b4][nb][i] = p;
          ps += p;
        }
      lsum[nb] += ps;  // lane-partial, summed over the column's 4 lanes in the epilogue
    }
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      bf16x8_t pa[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[nb][j] = (__bf16)sc[2 * t2][nb][j];
          pa[nb][4 + j] = (__bf16)sc[2 * t2 + 1][nb][j];
        }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const char* p0 = img + vofs[n] + 32 * t2 * RB;
        s16x4_t lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
        s16x4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * RB));
        const bf16x8_t vb = __builtin_bit_cast(
            bf16x8_t, s16x8_t{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]});
        o[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[0], vb, o[0][n], 0, 0, 0);
        o[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[1], vb, o[1][n], 0, 0, 0);
      }
    }
  };

  const int ntile = (hi - lo + 63) >> 6;
  issue(buf0, 0);
  for (int t = 0; t < ntile; t += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < ntile) issue(buf1, t + 1);
    compute(buf0, t);
    if (t + 1 >= ntile) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 2 < ntile) issue(buf0, t + 2);
    compute(buf1, t + 1);
  }

  // partials: O (unnormalised, v-scaled), running max M and sum L (log2 units)
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    float den = lsum[nb] + __shfl_xor(lsum[nb], 16, 64);
    den += __shfl_xor(den, 32, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cc = 4 * g + i;
      const float mc = __shfl(m[nb], cc, 64);
      const float lc = __shfl(den, cc, 64);
      const int mi = col_member(nb, cc);
      if (mi < nm) {
        const int b = members[m0 + mi];
        const int64_t pi = ((int64_t)b * Hq + col_head(nb)) * nslot + pslot0 + slot;
#pragma unroll
        for (int n = 0; n < NB; ++n) part_o[pi * D + 16 * n + c16] = o[nb][n][i] * vscale;
        if (c16 == 0) {
          part_ml[pi * 2] = mc;
          part_ml[pi * 2 + 1] = lc;
        }
      }
    }
  }
}

// Merge a sequence's partials: suffix splits [0, nact) and, with a shared
// prefix, the prefix kernel's slots [pslot0, pslot0 + pcount[b]).
template <int D>
__global__ __launch_bounds__(64) void decode_reduce_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_ml,
    const int* __restrict__ seq_lens, const int* __restrict__ sstart, const int* __restrict__ pcount,
    int Hq, int nsplit, int nslot, int split_size, const int* __restrict__ split_dev, int window,
    const float* __restrict__ sinks, uint16_t* __restrict__ out, int64_t out_stride) {
  const int hq = blockIdx.x, b = blockIdx.y;
  const int L = seq_lens[b];
  int start = window > 0 ? max(0, L - window) : 0;
  if (sstart) start = max(start, sstart[b]);
  if (split_dev) split_size = *split_dev;
  const int nact = min(nsplit, (L - start + split_size - 1) / split_size);
  const int np = pcount ? pcount[b] : 0;
  const int64_t base = ((int64_t)b * Hq + hq) * nslot;
  auto slot = [&](int s) { return s < nact ? s : nsplit + (s - nact); };
  const int ntot = nact + np;
  float M = NEG_INF;
  for (int s = 0; s < ntot; ++s) M = fmaxf(M, part_ml[(base + slot(s)) * 2]);
  float den = 0.f;
  for (int s = 0; s < ntot; ++s)
    den += exp2f(part_ml[(base + slot(s)) * 2] - M) * part_ml[(base + slot(s)) * 2 + 1];
  if (sinks) den += exp2f(sinks[hq] * 1.4426950408889634f - M);
  const float inv = 1.f / den;
  for (int d = threadIdx.x; d < D; d += 64) {
    float acc = 0.f;
    for (int s = 0; s < ntot; ++s)
      acc += exp2f(part_ml[(base + slot(s)) * 2] - M) * part_o[(base + slot(s)) * D + d];
    out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(acc * inv);
  }
}

}  // namespace

extern "C" int llmd_paged_decode(const void* q, int64_t q_stride, const void* kc, const void* vc,
                                 int64_t block_stride, int bs, const int* block_tables,
                                 int bt_stride, const int* seq_lens, int B, int Hq, int Hkv, int D,
                                 float scale, int window, const float* sinks, int split_size,
                                 int nsplit, void* out, int64_t out_stride, float* part_o,
                                 float* part_ml, int fp8, float k_scale, float v_scale,
                                 const int* sstart, const int* pcount, const int* members, const int* work,
                                 int nwork, int np, int nslot, const int* split_dev, hipStream_t st) {
  if (B == 0) return 0;
  const int G = Hq / Hkv;
  const int NG = (G + 15) / 16;
  const float scale_log2 = scale * k_scale * 1.4426950408889634f;
  const bool cascade = work != nullptr && nwork > 0;
  if (cascade && (G > 16 || 16 % G != 0 || np < 1 || np > 3)) return -2;
  // np 3: the LDS-DMA prefix kernel (bf16 cache, G 4 or 8, >= 8 keys per block)
  if (cascade && np == 3 && (fp8 || (G != 4 && G != 8) || bs < 8)) return -4;
  const int direct = (nsplit == 1 && !cascade) ? 1 : 0;
  if (!direct && nslot < nsplit) return -3;
  dim3 grid(nsplit, Hkv * NG, B), blk(NT);
  const size_t lds = (size_t)4 * 64 * D * 2;
  static const bool nt_env = [] {  // non-temporal K/V loads by default (LLMD_DECODE_NT=0 for A/B): with the
    const char* e = getenv("LLMD_DECODE_NT");  // nt weight stream, 70B decode 44.1 -> 43.5 ms/step
    return !(e && e[0] == '0');                 // (profiles/decode_nt_r4.txt)
  }();
  auto decode_nt = [] { return nt_env; };
#define LAUNCH(DD, F8)                                                                                       \
  do {                                                                                                       \
    if (cascade) {                                                                                           \
      if (np == 3 && !F8)                                                                                    \
        hipLaunchKernelGGL((shared_prefix_v2_kernel<DD>), dim3(Hkv, nwork), blk, 0, st, (const uint16_t*)q,  \
                           q_stride, (const uint16_t*)kc, (const uint16_t*)vc, block_stride, bs,             \
                           block_tables, bt_stride, members, work, Hq, G, scale_log2, nslot, nsplit, part_o, \
                           part_ml, v_scale);                                                                \
      else if (np == 1)                                                                                      \
        hipLaunchKernelGGL((shared_prefix_kernel<DD, F8, 1>), dim3(Hkv, nwork), blk, lds, st,               \
                           (const uint16_t*)q, q_stride, kc, vc, block_stride, bs, block_tables, bt_stride,  \
                           members, work, Hq, G, scale_log2, nslot, nsplit, part_o, part_ml, v_scale);               \
      else                                                                                                   \
        hipLaunchKernelGGL((shared_prefix_kernel<DD, F8, 2>), dim3(Hkv, nwork), blk, lds, st,               \
                           (const uint16_t*)q, q_stride, kc, vc, block_stride, bs, block_tables, bt_stride,  \
                           members, work, Hq, G, scale_log2, nslot, nsplit, part_o, part_ml, v_scale);               \
    }                                                                                                        \
    hipLaunchKernelGGL((decode_nt() ? paged_decode_kernel<DD, F8, true> : paged_decode_kernel<DD, F8, false>), \
                       grid, blk, lds, st, (const uint16_t*)q, q_stride, kc,                                 \
                       vc, block_stride, bs, block_tables, bt_stride, seq_lens, cascade ? sstart : nullptr,  \
                       Hq, Hkv, G, NG, scale_log2, window, sinks, split_size, split_dev,                     \
                       direct ? nsplit : nslot,                                                              \
                       direct, (uint16_t*)out, out_stride, part_o, part_ml, v_scale);                        \
    if (!direct)                                                                                             \
      hipLaunchKernelGGL(decode_reduce_kernel<DD>, dim3(Hq, B), dim3(64), 0, st, part_o, part_ml, seq_lens,  \
                         cascade ? sstart : nullptr, cascade ? pcount : nullptr, Hq, nsplit,                 \
                         direct ? nsplit : nslot, split_size, split_dev, window, sinks, (uint16_t*)out,       \
                         out_stride);                                                                        \
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
