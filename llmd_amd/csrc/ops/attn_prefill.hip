// Varlen causal prefill / chunked-prefill attention over the paged KV cache
// (SURVEY K02/K04). New tokens' K/V must already be in the cache (rope_cache).
//
// Work decomposition: a host-built list of items (seq, first query token of a
// 32*TPW-token block) x grid.y = (kv head, head group). A workgroup = 4 waves;
// wave w owns 32 query tokens of one query head, and the HPW heads handled by
// one workgroup all share the same KV head, so every K/V tile staged in LDS is
// reused by all 4 waves (GQA reuse) and - for G >= 4 - all waves share the same
// causal range (no imbalance).
//
// Per 64-key tile:
//   S^T[key][q] = K[key] . Q[q]   (keys on the MFMA M axis -> P lands lane-local
//                                  in the A-operand layout of the PV product)
//     K image: padded rows (D*2+16 B) -> ds_read_b128 conflict-free
//   O[q][dim] += P[q][key] . V[key][dim]
//     V image: XOR-swizzled rows, ds_read_b64_tr_b16 transposed reads
// K/V tiles are double-buffered; the next tile's global loads are issued before
// the current tile's MFMAs and written to LDS after the barrier (T14 split).
#include <cstdlib>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;
constexpr float NEG_INF = -__builtin_huge_valf();

__device__ __forceinline__ int rowoff(int g) { return 4 * (g >> 1) + 8 * (g & 1); }

template <int D>
__device__ __forceinline__ int vimg_off(int row, int ch) {
  if constexpr (D == 128) {
    const int sw = ((row & 3) << 2) | ((row >> 2) & 3);
    return row * 256 + 16 * (ch ^ sw);
  } else {
    const int sw = 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
    return row * 128 + 16 * (ch ^ sw);
  }
}
template <int D>
__device__ __forceinline__ int kimg_off(int row, int ch) {
  return row * (D * 2 + 16) + 16 * ch;
}

// fp8 (e4m3fn) caches: tiles are loaded packed (8 B per 8 elements) and widened
// to bf16 when written to LDS, so the LDS images and MFMAs are unchanged.
template <bool F8>
struct CacheReg {
  using T = u32x4_t;
};
template <>
struct CacheReg<true> {
  using T = u32x2_t;
};

template <int D, bool F8>
__global__ __launch_bounds__(NT, 2) void prefill_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const void* __restrict__ kc,
    const void* __restrict__ vc, int64_t block_stride, int bs,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len, const int* __restrict__ items,
    int Hq, int Hkv, int G, int HPW, float scale_log2, int window,
    const float* __restrict__ sinks, uint16_t* __restrict__ out, int64_t out_stride, float vscale) {
  using CR = typename CacheReg<F8>::T;
  constexpr int KS = D / 32, NB = D / 16, CPR = D / 8;
  constexpr int KIMG = 64 * (D * 2 + 16);
  constexpr int VIMG = 64 * D * 2;
  constexpr int LPT = 64 * CPR / NT;  // chunks per thread per tile (K and V each)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int seq = items[2 * blockIdx.x], qb = items[2 * blockIdx.x + 1];
  const int NHG = G / HPW;
  const int kvh = blockIdx.y / NHG, hg = blockIdx.y % NHG;
  const int TPW = 4 / HPW;  // token sub-blocks per workgroup
  const int qs = q_start[seq], ql = q_len[seq], ctx = ctx_len[seq];
  const int pbase = ctx - ql;  // position of query token 0
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);  // block size is a power of two (checked on the host)

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int head = kvh * G + hg * HPW + (w % HPW);
  const int tok0 = qb + (w / HPW) * 32;
  const int ntok = max(0, min(32, ql - tok0));
  const int p_lo = pbase + tok0, p_hi = pbase + tok0 + max(ntok, 1) - 1;

  // workgroup key range
  const int wg_tok_end = min(ql, qb + 32 * TPW);
  const int wg_p_lo = pbase + qb, wg_p_hi = pbase + wg_tok_end - 1;
  const int kmin = window > 0 ? max(0, wg_p_lo - window + 1) : 0;
  const int t_first = kmin >> 6, t_last = wg_p_hi >> 6;

  // Q fragments: B operand, [nb][s]
  bf16x8_t qf[2][KS];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int tk = tok0 + 16 * nb + c16;
    const uint16_t* qr = q + (int64_t)(qs + tk) * q_stride + (int64_t)head * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (tk < ql) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      qf[nb][s] = __builtin_bit_cast(bf16x8_t, v);
    }
  }

  float m[2] = {NEG_INF, NEG_INF}, lsum[2] = {0.f, 0.f};
  f32x4_t o[2][NB];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int n = 0; n < NB; ++n) o[nb][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- tile loader (registers)
  CR kr[LPT], vr[LPT];
  auto load_tile = [&](int t) {
    const int ts = t * 64;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int row = idx / CPR, ch = idx % CPR;
      int key = ts + row;
      key = key < ctx ? key : ctx - 1;
      const int phys = bt[key >> lbs];
      const int64_t off = (int64_t)phys * block_stride + head_off + (int64_t)(key & (bs - 1)) * D + ch * 8;
      if constexpr (F8) {
        kr[i] = *reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(kc) + off);
        vr[i] = *reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(vc) + off);
      } else {
        kr[i] = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(kc) + off);
        vr[i] = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(vc) + off);
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* kimg = smem + buf * (KIMG + VIMG);
    char* vimg = kimg + KIMG;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int row = idx / CPR, ch = idx % CPR;
      if constexpr (F8) {
        *reinterpret_cast<u32x4_t*>(kimg + kimg_off<D>(row, ch)) = fp8x8_to_bf16x8(kr[i]);
        *reinterpret_cast<u32x4_t*>(vimg + vimg_off<D>(row, ch)) = fp8x8_to_bf16x8(vr[i]);
      } else {
        *reinterpret_cast<u32x4_t*>(kimg + kimg_off<D>(row, ch)) = kr[i];
        *reinterpret_cast<u32x4_t*>(vimg + vimg_off<D>(row, ch)) = vr[i];
      }
    }
  };

  load_tile(t_first);
  int buf = 0;
  for (int t = t_first; t <= t_last; ++t) {
    store_tile(buf);
    __syncthreads();
    if (t < t_last) load_tile(t + 1);
    const int ts = t * 64;
    const bool active = ntok > 0 && ts <= p_hi && (window <= 0 || ts + 63 > p_lo - window);
    if (active) {
      const char* kimg = smem + buf * (KIMG + VIMG);
      const char* vimg = kimg + KIMG;
      // ---- S^T
      f32x4_t sc[4][2];
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) {
        const int row = 16 * b4 + rowoff(c16 >> 2) + (c16 & 3);
        f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bf16x8_t ka = *reinterpret_cast<const bf16x8_t*>(kimg + kimg_off<D>(row, 4 * s + g));
          a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[0][s], a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[1][s], a1, 0, 0, 0);
        }
        sc[b4][0] = a0;
        sc[b4][1] = a1;
      }
      // ---- mask (only tiles that touch the diagonal / window edge) + online softmax.
      // Scores stay raw; the row max m is kept in scaled log2 units and
      // p = exp2(s*scale_log2 - m) is one FMA + v_exp. Lazy rescaling: m only
      // moves when some row's max grows by more than 8 (p <= 2^8 stays exact
      // enough in bf16/fp32), so O/l rescales are rare after the first tiles.
      const bool need_mask = (ts + 63 > p_lo) || (window > 0 && ts <= p_hi - window);
      if (need_mask) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const int qp = p_lo + 16 * nb + c16;
#pragma unroll
          for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int key = ts + 16 * b4 + rowoff(g) + i;
              bool ok = key <= qp;
              if (window > 0) ok = ok && key > qp - window;
              sc[b4][nb][i] = ok ? sc[b4][nb][i] : NEG_INF;
            }
        }
      }
      float mt[2];
      bool grow = false;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        float mx = NEG_INF;
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[b4][nb][i]);
        mt[nb] = mx * scale_log2;  // lane-local (see prefill_v2_kernel)
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
        // fully masked rows so far keep m = -inf: their p must be 0, not exp2(nan)
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
        lsum[nb] += ps;  // lane-partial, reduced in the epilogue
      }
      // ---- O += P V
      const int qq = c16 >> 2, pp = c16 & 3;
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
          const int r0 = 32 * t2 + rowoff(g) + qq;
          const int ch = 2 * n + (pp >> 1);
          const int a0 = vimg_off<D>(r0, ch) + 8 * (pp & 1);
          const int a1 = vimg_off<D>(r0 + 16, ch) + 8 * (pp & 1);
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(vimg + a0));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(vimg + a1));
          const bf16x8_t vb = __builtin_bit_cast(
              bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
          o[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[0], vb, o[0][n], 0, 0, 0);
          o[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[1], vb, o[1][n], 0, 0, 0);
        }
      }
    }
    buf ^= 1;
  }

  // ---- epilogue: rows of O are q tokens 16*nb + 4g + i; their m/l live in lane 4g+i
  if (ntok == 0) return;
  const float sink = sinks ? sinks[head] * 1.4426950408889634f : NEG_INF;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    float den = lsum[nb] + __shfl_xor(lsum[nb], 16, 64);
    den += __shfl_xor(den, 32, 64);
    if (sinks) den += exp2f(sink - (m[nb] == NEG_INF ? 0.f : m[nb]));
    const float inv = den > 0.f ? vscale / den : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float f = __shfl(inv, 4 * g + i, 64);
      const int tk = tok0 + 16 * nb + 4 * g + i;
      if (tk < ql) {
        uint16_t* orow = out + (int64_t)(qs + tk) * out_stride + (int64_t)head * D;
#pragma unroll
        for (int n = 0; n < NB; ++n) orow[16 * n + c16] = f2bf(o[nb][n][i] * f);
      }
    }
  }
}

// ---------------------------------------------------------------- v2 (bf16 cache, D = 64/128, block >= 16)
// Same work decomposition and math as prefill_kernel; the tiles move
// global -> LDS with global_load_lds_dwordx4 (no VGPR staging, no ds_write),
// one vmcnt + barrier per tile, double-buffered. Images are unpadded 256-B rows
// with per-row XOR swizzles of the 16-B chunk, applied on the DMA source side:
//   K: slot = c ^ pk(r), pk(r) = ((r >> 1) & 7) | ((r & 1) << 3): every
//      ds_read_b128 lane group of the S^T A-operand reads covers 16 distinct
//      16-B bank slots (rows {0-3,12-15} vs {4-11} at chunks 4s+g / 4s+g^1).
//   V: slot = c ^ pv(r), pv(r) = 2 ((r & 3) | (((r >> 3) & 1) << 2)): the 32-lane
//      ds_read_b64_tr_b16 groups (rows {0-3,8-11} / {4-7,12-15}, chunk pairs
//      2n, 2n+1) hit 32 distinct 8-B slots.
//   D = 64 (128-B rows, 8 chunks; odd rows shift banks by half a bank row):
//      K and V both use (r & 2) | ((r >> 1) & 4), found by the same exhaustive
//      search as the MLA latent tile, which has the same bank geometry.
// All LDS reads are a per-lane register + an immediate (buffer, key block, dim block).
template <int D>
__device__ __forceinline__ int p2_pk(int r) {
  if constexpr (D == 128) return ((r >> 1) & 7) | ((r & 1) << 3);
  else return (r & 2) | ((r >> 1) & 4);
}
template <int D>
__device__ __forceinline__ int p2_pv(int r) {
  if constexpr (D == 128) return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
  else return (r & 2) | ((r >> 1) & 4);
}

// V (round-4 A/B switch): bit 0 = K/V fragment reads ring-pipelined with a sched_barrier
// per step, bit 1 = LDS-DMA from asm (glds16) instead of the builtin
// (round 6) bit 4 = row sums kept in scalar f32 adds: hipcc SLP-packs the two query blocks' sums
// into v_pk_add_f32, which beside MFMAs costs ~13 cycles more per instruction than two v_add_f32
// (MI355X_MICROARCH 'price of one filler beside MFMAs'); bit 5 = whole tiles DMA'd through a
// per-tile buffer descriptor (scalar base, 32-bit per-lane offsets) instead of 64-bit per-lane
// addresses (the v_lshl_add_u64 of every piece); bit 6 = the causal / window mask behind a scalar
// branch (see compute()). The loop is issue-bound (profiles/attn_prefill_v2_variants_r6.txt), so
// bits 7 / 8 take VALU work per score away: bit 7 = Q pre-scaled by scale * log2(e) at load and the
// S^T accumulators started at -m (the running row max, one broadcast register per query block):
// the MFMA yields S scale - m, and p = exp2 of it without the per-score v_fma; bit 8 = row sums on
// the matrix pipe: P . ones (4 extra 16x16x32 MFMAs per tile, accumulators in O's layout) instead of
// 32 v_add_f32 per lane and tile, and no cross-lane sum in the epilogue
template <int D, int V = 3>
__global__ __launch_bounds__(NT, 2) void prefill_v2_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int64_t block_stride, int bs,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len, const int* __restrict__ items,
    int Hq, int Hkv, int G, int HPW, float scale_log2, int window,
    const float* __restrict__ sinks, uint16_t* __restrict__ out, int64_t out_stride, float vscale, int xcd) {
  constexpr int KS = D / 32, NB = D / 16, RB = 2 * D;  // row bytes
  constexpr int P2_IMG = 64 * RB;                       // one 64-key bf16 image
  constexpr int NI = 64 * (D / 8) / 64;                 // DMA wave-instructions per image (16 / 8)
  __shared__ __attribute__((aligned(1024))) char buf0[2 * P2_IMG];  // K | V of even tiles
  __shared__ __attribute__((aligned(1024))) char buf1[2 * P2_IMG];  // K | V of odd tiles

  // xcd: the dispatcher deals workgroups round-robin over the 8 XCDs; remap so
  // each XCD runs a contiguous (head group, item) range - one KV head's K/V
  // (5000 tokens: 2.5 MB) stays in that XCD's 4 MB L2 instead of every XCD
  // streaming all heads' tiles. Measured (profiles/attn_prefill_r2_lanelocal.txt):
  // ISL 5000 776 -> 833 TF/s, 8k 932 -> 1016; a one-wave grid (5000 x 512
  // chunk, 256 workgroups) loses 2 %, so the host enables it from 1024 workgroups
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int l = xcd_remap(by * gridDim.x + bx, gridDim.x * gridDim.y);
    bx = l % gridDim.x;
    by = l / gridDim.x;
  }
  const int seq = items[2 * bx], qb = items[2 * bx + 1];
  const int NHG = G / HPW;
  const int kvh = by / NHG, hg = by % NHG;
  const int TPW = 4 / HPW;
  const int qs = q_start[seq], ql = q_len[seq], ctx = ctx_len[seq];
  const int pbase = ctx - ql;
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int head = kvh * G + hg * HPW + (w % HPW);
  const int tok0 = qb + (w / HPW) * 32;
  const int ntok = max(0, min(32, ql - tok0));
  const int p_lo = pbase + tok0, p_hi = pbase + tok0 + max(ntok, 1) - 1;
  const int wg_tok_end = min(ql, qb + 32 * TPW);
  const int wg_p_lo = pbase + qb, wg_p_hi = pbase + wg_tok_end - 1;
  const int kmin = window > 0 ? max(0, wg_p_lo - window + 1) : 0;
  const int t_first = kmin >> 6, t_last = wg_p_hi >> 6;

  bf16x8_t qf[2][KS];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int tk = tok0 + 16 * nb + c16;
    const uint16_t* qr = q + (int64_t)(qs + tk) * q_stride + (int64_t)head * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (tk < ql) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      qf[nb][s] = __builtin_bit_cast(bf16x8_t, v);
      if constexpr ((V & 128) != 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[nb][s][e] = (__bf16)((float)qf[nb][s][e] * scale_log2);
      }
    }
  }
  float m[2] = {NEG_INF, NEG_INF}, lsum[2] = {0.f, 0.f};
  f32x4_t o[2][NB];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int n = 0; n < NB; ++n) o[nb][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // bit 7: -m (0 while no score seen) broadcast, the S^T accumulators' start; bit 8: row sums in O's layout
  f32x4_t cm[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  f32x4_t ls[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  constexpr bool RELS = (V & 128) != 0, MSUM = (V & 256) != 0;
  const float sl2 = RELS ? 1.f : scale_log2;  // scale of the scores the MFMA yields (bit 7: pre-applied)

  // DMA: NI K + NI V wave-instructions of 1 KB (1024 / RB rows); wave w issues
  // j = w + 4i. The per-lane source offsets inside a 64-row tile are constant
  // (row * RB + swizzled 16-B slot), so a tile costs one scalar base (block
  // table lookup) plus a VGPR offset per load (global_load_lds saddr+voffset,
  // -12 % VALU instructions); only a sequence's last, partial tile clamps rows
  // (its V rows past the end must stay finite: P = 0 there, but 0 * NaN would
  // poison O).
  const int ws = __builtin_amdgcn_readfirstlane(w);
  uint32_t koff[4], voff[4];  // NI / 4 used; fixed size: a template-sized array read by the DMA lambda loses the launch stub
#pragma unroll
  for (int i = 0; i < NI / 4; ++i) {
    const int u = 64 * (w + 4 * i) + lane;
    const int row = u / (D / 8), sl = u % (D / 8);
    koff[i] = (uint32_t)(row * RB + 16 * (sl ^ p2_pk<D>(row)));
    voff[i] = (uint32_t)(row * RB + 16 * (sl ^ p2_pv<D>(row)));
  }
  auto dma = [&](const char* src, char* dst) {
    if constexpr (V & 2) glds16(src, lds_addr(dst));
    else __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                          (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  auto issue = [&](char* base, int t) {
    const int ts = t * 64;
    LLMD_DCHECK(ts < ctx && bt[ts >> lbs] >= 0 && ctx <= bt_stride * bs);
    const int64_t tb = 2 * ((int64_t)bt[ts >> lbs] * block_stride + head_off + (int64_t)(ts & (bs - 1)) * D);
    const char* kb = reinterpret_cast<const char*>(kc) + tb;
    const char* vb = reinterpret_cast<const char*>(vc) + tb;
    const int rlim = ctx - 1 - ts;
    if (rlim >= 63 && bs >= 64) {
      if constexpr ((V & 32) != 0) {
        const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)kb, 0, 64 * RB, 0x00020000);
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)vb, 0, 64 * RB, 0x00020000);
#pragma unroll
        for (int i = 0; i < NI / 4; ++i) {
          char* dst = base + 1024 * (ws + 4 * i);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)dst, 16, koff[i], 0, 0, 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(dst + P2_IMG), 16,
                                                   voff[i], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NI / 4; ++i) {
          char* dst = base + 1024 * (ws + 4 * i);
          dma(kb + koff[i], dst);
          dma(vb + voff[i], dst + P2_IMG);
        }
      }
    } else if (rlim >= 63) {
      // blocks of 16 / 32 keys: a wave-instruction's RPI rows sit in one block
      // (bs >= RPI), so one scalar block-table lookup per instruction
      constexpr int RPI = 1024 / RB;
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        const int r0 = RPI * (ws + 4 * i);
        const int key0 = ts + r0;
        const int64_t ib = 2 * ((int64_t)bt[key0 >> lbs] * block_stride + head_off + (int64_t)(key0 & (bs - 1)) * D) -
                           (int64_t)r0 * RB;
        char* dst = base + 1024 * (ws + 4 * i);
        dma(reinterpret_cast<const char*>(kc) + ib + koff[i], dst);
        dma(reinterpret_cast<const char*>(vc) + ib + voff[i], dst + P2_IMG);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        const int u = 64 * (w + 4 * i) + lane;
        const int row = u / (D / 8), sl = u % (D / 8);
        const int key = ts + min(row, rlim);
        // row offset from the tile base when the tile is one block, else the key's own block
        const int64_t ro = bs >= 64 ? (int64_t)min(row, rlim) * RB
                                    : 2 * ((int64_t)bt[key >> lbs] * block_stride + head_off +
                                           (int64_t)(key & (bs - 1)) * D) - tb;
        char* dst = base + 1024 * (ws + 4 * i);
        dma(kb + ro + 16 * (sl ^ p2_pk<D>(row)), dst);
        dma(vb + ro + 16 * (sl ^ p2_pv<D>(row)), dst + P2_IMG);
      }
    }
  };
  // per-lane LDS offsets (see the header): K rows 16 b4 + srow, chunk 4s + g;
  // V rows 32 t2 + vrow (+16), chunk 2n + (pp >> 1), half pp & 1
  const int qq = c16 >> 2, pp = c16 & 3;
  const int srow = rowoff(c16 >> 2) + (c16 & 3), kp = p2_pk<D>(srow);
  int kofs[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) kofs[s] = srow * RB + 16 * ((4 * s + g) ^ kp);
  const int vrow = rowoff(g) + qq, vp = p2_pv<D>(vrow);
  int vofs[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) vofs[n] = P2_IMG + vrow * RB + 16 * ((2 * n + (pp >> 1)) ^ vp) + 8 * (pp & 1);

  auto compute = [&](const char* img, int t) {
    const int ts = t * 64;
    const bool active = ntok > 0 && ts <= p_hi && (window <= 0 || ts + 63 > p_lo - window);
    if (!active) return;
    // S^T: K fragment j = KS b4 + s, read PF ahead of its two MFMAs (a ring with a
    // sched_barrier per step: hipcc's own schedule hoists every read and waits lgkmcnt(0))
    constexpr int PF = (V & 4) ? 6 : 4;  // fragments read ahead (V bit 2: 6)
    auto kread = [&](int j) {
      return *reinterpret_cast<const bf16x8_t*>(img + kofs[j % KS] + (j / KS) * 16 * RB);
    };
    // PV: V fragment j = NB t2 + n (two transposed reads), PF ahead of its two MFMAs
    auto vread = [&](int j) {
      const char* p0 = img + vofs[j % NB] + 32 * (j / NB) * RB;
      s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
      s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * RB));
      return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    };
    bf16x8_t vr[PF];
    f32x4_t sc[4][2];
    bf16x8_t kr[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) kr[j] = kread(j);
    if constexpr (V & 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      f32x4_t a0 = cm[0], a1 = cm[1];  // zeros unless bit 7
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int j = KS * b4 + s;
        const bf16x8_t ka = kr[j % PF];
        if (j + PF < 4 * KS) kr[j % PF] = kread(j + PF);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[0][s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[1][s], a1, 0, 0, 0);
        if constexpr (V & 1) __builtin_amdgcn_sched_barrier(0);
      }
      sc[b4][0] = a0;
      sc[b4][1] = a1;
    }
    if constexpr (V & 8) {  // the first V fragments load under the mask + softmax (V bit 3)
#pragma unroll
      for (int j = 0; j < PF; ++j) vr[j] = vread(j);
    }
    bool need_mask = (ts + 63 > p_lo) || (window > 0 && ts <= p_hi - window);
    if constexpr ((V & 64) != 0) need_mask = __builtin_amdgcn_readfirstlane((int)need_mask) != 0;
    if (need_mask) {
      // bit 6: a real (scalar) branch - without the asm fence hipcc if-converts the mask into
      // ~290 selects / compares executed on EVERY tile, not just the diagonal and window-edge ones
      if constexpr ((V & 64) != 0) asm volatile("" ::: "memory");
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int qp = p_lo + 16 * nb + c16;
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = ts + 16 * b4 + rowoff(g) + i;
            bool ok = key <= qp;
            if (window > 0) ok = ok && key > qp - window;
            sc[b4][nb][i] = ok ? sc[b4][nb][i] : NEG_INF;
          }
      }
    }
    // lane-local maxima decide whether any row of the wave needs a rescale
    // (a row max can only exceed m + 8 if one of its 4 lanes' does): the
    // cross-lane reductions run only then, not every tile
    float mt[2];
    bool grow = false;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float mx = NEG_INF;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[b4][nb][i]);
      if constexpr (RELS) {  // scores relative to msub (0 while m = -inf): absolute max = mx + msub
        const float msub = (m[nb] == NEG_INF) ? 0.f : m[nb];
        mt[nb] = mx + msub;
      } else {
        mt[nb] = mx * scale_log2;
      }
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
        lsum[nb] *= alpha[nb];  // per-lane partial sums, same factor on the row's 4 lanes
        if constexpr (RELS) {   // rebase this tile's relative scores and the next tiles' start
          const float sold = (m[nb] == NEG_INF) ? 0.f : m[nb], snew = (mnew == NEG_INF) ? 0.f : mnew;
          const float d = sold - snew;
#pragma unroll
          for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
            for (int i = 0; i < 4; ++i) sc[b4][nb][i] += d;
          cm[nb] = f32x4_t{-snew, -snew, -snew, -snew};
        }
        m[nb] = mnew;
      }
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = __shfl(alpha[nb], 4 * g + i, 64);
#pragma unroll
          for (int n = 0; n < NB; ++n) o[nb][n][i] *= a;
          if constexpr (MSUM) ls[nb][i] *= a;
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
          const float p = RELS ? __builtin_amdgcn_exp2f(sc[b4][nb][i])
                               : __builtin_amdgcn_exp2f(fmaf(sc[b4][nb][i], sl2, -msub));
          sc[b4][nb][i] = p;
          if constexpr (!MSUM) {
            ps += p;
            if constexpr ((V & 16) != 0) asm volatile("" : "+v"(ps));  // no SLP packing across nb
          }
        }
      if constexpr (!MSUM) lsum[nb] += ps;  // lane-partial: summed over the row's 4 lanes once, in the epilogue
    }
    bf16x8_t pa[2][2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[t2][nb][j] = (__bf16)sc[2 * t2][nb][j];
          pa[t2][nb][4 + j] = (__bf16)sc[2 * t2 + 1][nb][j];
        }
    if constexpr (MSUM) {  // row sums of P on the matrix pipe: P . ones, rows in O's layout
      const bf16x8_t ones = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                             (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        ls[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[t2][0], ones, ls[0], 0, 0, 0);
        ls[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[t2][1], ones, ls[1], 0, 0, 0);
      }
    }
    if constexpr (!(V & 8)) {
#pragma unroll
      for (int j = 0; j < PF; ++j) vr[j] = vread(j);
    }
    if constexpr (V & 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) {
      const int t2 = j / NB, n = j % NB;
      const bf16x8_t vb = vr[j % PF];
      if (j + PF < 2 * NB) vr[j % PF] = vread(j + PF);
      o[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[t2][0], vb, o[0][n], 0, 0, 0);
      o[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[t2][1], vb, o[1][n], 0, 0, 0);
      if constexpr (V & 1) __builtin_amdgcn_sched_barrier(0);
    }
  };

  issue(buf0, t_first);
  for (int t = t_first; t <= t_last; t += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 <= t_last) issue(buf1, t + 1);
    compute(buf0, t);
    if (t + 1 > t_last) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 2 <= t_last) issue(buf0, t + 2);
    compute(buf1, t + 1);
  }

  if (ntok == 0) return;
  const float sink = sinks ? sinks[head] * 1.4426950408889634f : NEG_INF;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    float den = lsum[nb] + __shfl_xor(lsum[nb], 16, 64);
    den += __shfl_xor(den, 32, 64);
    if (sinks) den += exp2f(sink - (m[nb] == NEG_INF ? 0.f : m[nb]));
    const float inv = den > 0.f ? vscale / den : 0.f;
    float mrow[4];  // bit 8: the running max of O's row 4 g + i (m is kept per query column c16)
#pragma unroll
    for (int i = 0; i < 4; ++i) mrow[i] = MSUM ? __shfl(m[nb], 4 * g + i, 64) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float f = __shfl(inv, 4 * g + i, 64);
      if constexpr (MSUM) {
        float d = ls[nb][i];
        if (sinks) d += exp2f(sink - (mrow[i] == NEG_INF ? 0.f : mrow[i]));
        f = d > 0.f ? vscale / d : 0.f;
      }
      const int tk = tok0 + 16 * nb + 4 * g + i;
      if (tk < ql) {
        uint16_t* orow = out + (int64_t)(qs + tk) * out_stride + (int64_t)head * D;
#pragma unroll
        for (int n = 0; n < NB; ++n) orow[16 * n + c16] = f2bf(o[nb][n][i] * f);
      }
    }
  }
}

// ---------------------------------------------------------------- v3 (bf16 cache, D = 128, block >= 64, G % 4 == 0)
// One 4-wave workgroup per CU (512 registers per wave) runs 4 query heads of a
// GQA group x 64 query tokens; each wave owns one head x 4 token blocks of 16,
// so every K fragment (S^T A operand) and every V fragment (PV B operand) read
// from LDS feeds four MFMAs (v2: two) and each K/V tile serves 256 query rows.
// O (4 x 8 f32x4 = 128 accumulators) lives in the literal AGPRs a[0:127],
// touched only by the generated asm of prefill_v3_agpr.inc (gen_prefill_v3.py);
// scores accumulate in VGPRs through asm MFMAs; K and V fragments are read 4
// steps ahead with a sched_barrier per step; the LDS-DMA is issued from asm
// (glds16) so hipcc's waitcnt pass keeps counted lgkmcnt(N) waits. Same tile
// images, swizzles, masking, lazy rescale and sinks as v2.
#include "prefill_v3_agpr.inc"

__device__ __forceinline__ void pf3_mfma4(f32x4_t& s0, f32x4_t& s1, f32x4_t& s2, f32x4_t& s3, const bf16x8_t& k,
                                          const bf16x8_t& q0, const bf16x8_t& q1, const bf16x8_t& q2,
                                          const bf16x8_t& q3, bool first) {
  if (first) {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %4, %5, 0\n\t"
        "v_mfma_f32_16x16x32_bf16 %1, %4, %6, 0\n\t"
        "v_mfma_f32_16x16x32_bf16 %2, %4, %7, 0\n\t"
        "v_mfma_f32_16x16x32_bf16 %3, %4, %8, 0"
        : "=&v"(s0), "=&v"(s1), "=&v"(s2), "=&v"(s3)
        : "v"(k), "v"(q0), "v"(q1), "v"(q2), "v"(q3));
  } else {
    asm volatile(
        "v_mfma_f32_16x16x32_bf16 %0, %4, %5, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %1, %4, %6, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %2, %4, %7, %2\n\t"
        "v_mfma_f32_16x16x32_bf16 %3, %4, %8, %3"
        : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3)
        : "v"(k), "v"(q0), "v"(q1), "v"(q2), "v"(q3));
  }
}

__global__ __launch_bounds__(NT, 1) void prefill_v3_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int64_t block_stride, int bs,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len, const int* __restrict__ items,
    int Hq, int Hkv, int G, float scale_log2, int window, const float* __restrict__ sinks,
    uint16_t* __restrict__ out, int64_t out_stride, float vscale, int xcd) {
  constexpr int D = 128, KS = D / 32, NB = D / 16, RB = 2 * D;
  constexpr int P2_IMG = 64 * RB;  // one 64-key bf16 image (16 KB)
  constexpr int NI = 64 * (D / 8) / 64;  // 16 DMA wave-instructions per image
  __shared__ __attribute__((aligned(1024))) char buf0[2 * P2_IMG];  // K | V of even tiles
  __shared__ __attribute__((aligned(1024))) char buf1[2 * P2_IMG];  // K | V of odd tiles

  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int l = xcd_remap(by * gridDim.x + bx, gridDim.x * gridDim.y);
    bx = l % gridDim.x;
    by = l / gridDim.x;
  }
  const int seq = items[2 * bx], tok0 = items[2 * bx + 1];
  const int NHG = G / 4;
  const int kvh = by / NHG, hg = by % NHG;
  const int qs = q_start[seq], ql = q_len[seq], ctx = ctx_len[seq];
  const int pbase = ctx - ql;
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, g = lane >> 4,
            c16 = lane & 15;
  const int head = kvh * G + hg * 4 + w;
  const int ntok = max(0, min(64, ql - tok0));
  const int p_lo = pbase + tok0, p_hi = pbase + tok0 + max(ntok, 1) - 1;
  const int kmin = window > 0 ? max(0, p_lo - window + 1) : 0;
  const int t_first = kmin >> 6, t_last = p_hi >> 6;

  bf16x8_t qf[4][KS];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int tk = tok0 + 16 * nb + c16;
    const uint16_t* qr = q + (int64_t)(qs + tk) * q_stride + (int64_t)head * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (tk < ql) v = *reinterpret_cast<const u32x4_t*>(qr + (4 * s + g) * 8);
      qf[nb][s] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  float m[4] = {NEG_INF, NEG_INF, NEG_INF, NEG_INF}, lsum[4] = {0.f, 0.f, 0.f, 0.f};
  PF3_ZERO_ACC();  // O = a[0:127]

  uint32_t koff[NI / 4], voff[NI / 4];
#pragma unroll
  for (int i = 0; i < NI / 4; ++i) {
    const int u = 64 * (w + 4 * i) + lane;
    const int row = u / (D / 8), sl = u % (D / 8);
    koff[i] = (uint32_t)(row * RB + 16 * (sl ^ p2_pk<D>(row)));
    voff[i] = (uint32_t)(row * RB + 16 * (sl ^ p2_pv<D>(row)));
  }
  auto issue = [&](char* base, int t) {
    const int ts = t * 64;
    LLMD_DCHECK(ts < ctx && bt[ts >> lbs] >= 0 && ctx <= bt_stride * bs);
    const int64_t tb = 2 * ((int64_t)bt[ts >> lbs] * block_stride + head_off + (int64_t)(ts & (bs - 1)) * D);
    const char* kb = reinterpret_cast<const char*>(kc) + tb;
    const char* vb = reinterpret_cast<const char*>(vc) + tb;
    const int rlim = ctx - 1 - ts;
    const unsigned lk = lds_addr(base) + 1024 * w, lv = lk + P2_IMG;
    if (rlim >= 63) {
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        glds16(kb + koff[i], lk + 4096 * i);
        glds16(vb + voff[i], lv + 4096 * i);
      }
    } else {
      // a sequence's last, partial tile: rows past the end re-read the last key (finite V)
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        int ln = lane;  // opaque: recomputed here, not hoisted
        asm volatile("" : "+v"(ln));
        const int u = 64 * (w + 4 * i) + ln;
        const int row = u / (D / 8), sl = u % (D / 8);
        const int64_t ro = (int64_t)min(row, rlim) * RB;
        glds16(kb + ro + 16 * (sl ^ p2_pk<D>(row)), lk + 4096 * i);
        glds16(vb + ro + 16 * (sl ^ p2_pv<D>(row)), lv + 4096 * i);
      }
    }
  };
  const int qq = c16 >> 2, pp = c16 & 3;
  const int srow = rowoff(c16 >> 2) + (c16 & 3), kp = p2_pk<D>(srow);
  int kofs[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) kofs[s] = srow * RB + 16 * ((4 * s + g) ^ kp);
  const int vrow = rowoff(g) + qq, vp = p2_pv<D>(vrow);
  int vofs[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) vofs[n] = P2_IMG + vrow * RB + 16 * ((2 * n + (pp >> 1)) ^ vp) + 8 * (pp & 1);

  auto compute = [&](const char* img, int t) {
    const int ts = t * 64;
    const bool active = ntok > 0 && ts <= p_hi && (window <= 0 || ts + 63 > p_lo - window);
    if (!active) return;
    auto kread = [&](int j) {
      return *reinterpret_cast<const bf16x8_t*>(img + kofs[j % KS] + (j / KS) * 16 * RB);
    };
    auto vread = [&](int j) {
      const char* p0 = img + vofs[j % NB] + 32 * (j / NB) * RB;
      s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
      s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * RB));
      return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    };
    // ---- S^T[key][token] for the 4 token blocks: K fragment j = KS b4 + s
    f32x4_t sc[4][4];  // [b4][nb]
    bf16x8_t kr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) kr[j] = kread(j);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int j = KS * b4 + s;
        const bf16x8_t ka = kr[j & 3];
        if (j + 4 < 4 * KS) kr[j & 3] = kread(j + 4);
        pf3_mfma4(sc[b4][0], sc[b4][1], sc[b4][2], sc[b4][3], ka, qf[0][s], qf[1][s], qf[2][s], qf[3][s], s == 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // score MFMAs (asm) -> VALU reads
    __builtin_amdgcn_sched_barrier(0);
    const bool need_mask = (ts + 63 > p_lo) || (window > 0 && ts <= p_hi - window);
    if (need_mask) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int qp = p_lo + 16 * nb + c16;
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = ts + 16 * b4 + rowoff(g) + i;
            bool ok = key <= qp;
            if (window > 0) ok = ok && key > qp - window;
            sc[b4][nb][i] = ok ? sc[b4][nb][i] : NEG_INF;
          }
      }
    }
    float mt[4];
    bool grow = false;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      float mx = NEG_INF;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[b4][nb][i]);
      mt[nb] = mx * scale_log2;
      grow = grow || (mt[nb] > m[nb] + 8.f);
    }
    if (__ballot(grow) != 0) {  // wave-uniform, rare after the first tiles
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        float mx = fmaxf(mt[nb], __shfl_xor(mt[nb], 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[nb], mx);
        const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m[nb] - mnew);
        lsum[nb] *= alpha;
        m[nb] = mnew;
        const float a0 = __shfl(alpha, 4 * g, 64), a1 = __shfl(alpha, 4 * g + 1, 64),
                    a2 = __shfl(alpha, 4 * g + 2, 64), a3 = __shfl(alpha, 4 * g + 3, 64);
        if (nb == 0) {
          PF3_RESCALE0(a0, a1, a2, a3);
        } else if (nb == 1) {
          PF3_RESCALE1(a0, a1, a2, a3);
        } else if (nb == 2) {
          PF3_RESCALE2(a0, a1, a2, a3);
        } else {
          PF3_RESCALE3(a0, a1, a2, a3);
        }
      }
    }
    bf16x8_t pa[2][4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
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
      lsum[nb] += ps;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[t2][nb][j] = (__bf16)sc[2 * t2][nb][j];
          pa[t2][nb][4 + j] = (__bf16)sc[2 * t2 + 1][nb][j];
        }
    }
    // ---- O[token][dim] += P[token][key] . V[key][dim]: V fragment j = NB t2 + n feeds the 4 token blocks
    bf16x8_t vr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) vr[j] = vread(j);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1" ::: "memory");  // pa (VALU) -> asm MFMA operand
    __builtin_amdgcn_sched_barrier(0);
    PF3_PV_BLOCK
  };

  issue(buf0, t_first);
  for (int t = t_first; t <= t_last; t += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 <= t_last) issue(buf1, t + 1);
    compute(buf0, t);
    if (t + 1 > t_last) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 2 <= t_last) issue(buf0, t + 2);
    compute(buf1, t + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA left in flight at exit

  if (ntok == 0) return;
  PF3_DRAIN();
  const float sink = sinks ? sinks[head] * 1.4426950408889634f : NEG_INF;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    float den = lsum[nb] + __shfl_xor(lsum[nb], 16, 64);
    den += __shfl_xor(den, 32, 64);
    if (sinks) den += exp2f(sink - (m[nb] == NEG_INF ? 0.f : m[nb]));
    const float inv = den > 0.f ? vscale / den : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x[NB];
      if (nb == 0) {
        if (i == 0) { PF3_READ_0_0(x) } else if (i == 1) { PF3_READ_0_1(x) } else if (i == 2) { PF3_READ_0_2(x) } else { PF3_READ_0_3(x) }
      } else if (nb == 1) {
        if (i == 0) { PF3_READ_1_0(x) } else if (i == 1) { PF3_READ_1_1(x) } else if (i == 2) { PF3_READ_1_2(x) } else { PF3_READ_1_3(x) }
      } else if (nb == 2) {
        if (i == 0) { PF3_READ_2_0(x) } else if (i == 1) { PF3_READ_2_1(x) } else if (i == 2) { PF3_READ_2_2(x) } else { PF3_READ_2_3(x) }
      } else {
        if (i == 0) { PF3_READ_3_0(x) } else if (i == 1) { PF3_READ_3_1(x) } else if (i == 2) { PF3_READ_3_2(x) } else { PF3_READ_3_3(x) }
      }
      const float f = __shfl(inv, 4 * g + i, 64);
      const int tk = tok0 + 16 * nb + 4 * g + i;
      if (tk < ql) {
        uint16_t* orow = out + (int64_t)(qs + tk) * out_stride + (int64_t)head * D;
#pragma unroll
        for (int n = 0; n < NB; ++n) orow[16 * n + c16] = f2bf(x[n] * f);
      }
    }
  }
}


// ---------------------------------------------------------------- v4 (bf16 cache, D = 128): 32x32x16 MFMAs
// The work decomposition, items, K/V tiles and the double-buffered LDS-DMA ring of v2; the two
// products run on v_mfma_f32_32x32x16_bf16. An MFMA holds its SIMD's vector issue for 8 of its 32
// cycles (16x16x32: 8 of 16), so per MFMA-cycle there is three times the room for the softmax
// VALU and the LDS reads that share the issue port (MI355X_MICROARCH 'vector-instruction ISSUE
// cost'; v2 is issue-bound beside its MFMAs).
//   S^T[key][q] = K . Q^T: A = 32 K rows (ds_read_b128), B = the wave's 32 queries (registers);
//     lane l holds query l & 31's scores of keys (r & 3) + 8 (r >> 2) + 4 (l >> 5) of a 32-key
//     block (r = 0..15): row max and sum are lane-local plus one permlane32_swap.
//   O^T[d][q] += V^T . P^T: P^T is S^T's accumulator used in place as the B operand (cvt_pk per
//     register pair; its k order is the accumulator's permuted key order), A = V^T read with two
//     ds_read_b64_tr_b16 per fragment in that same key order.
// O^T's column is the query, so the online-softmax rescale is a lane-local multiply.
// Images: 256-B rows, 16-B chunk ch of row r at slot ch ^ (((r & 3) << 2) | ((r >> 2) & 3))
// (vimg_off<128>): conflict-free for the 32-row b128 reads and the transposed reads alike.
__device__ __forceinline__ int p4_sw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

template <int V4 = 1>
__global__ __launch_bounds__(NT, 2) void prefill_v4_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int64_t block_stride, int bs,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ q_start,
    const int* __restrict__ q_len, const int* __restrict__ ctx_len, const int* __restrict__ items,
    int Hq, int Hkv, int G, int HPW, float scale_log2, int window,
    const float* __restrict__ sinks, uint16_t* __restrict__ out, int64_t out_stride, float vscale, int xcd) {
  constexpr int D = 128, RB = 256, IMG = 64 * RB, NI = 16;
  __shared__ __attribute__((aligned(1024))) char buf0[2 * IMG];  // K | V of even tiles
  __shared__ __attribute__((aligned(1024))) char buf1[2 * IMG];  // K | V of odd tiles

  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int l = xcd_remap(by * gridDim.x + bx, gridDim.x * gridDim.y);
    bx = l % gridDim.x;
    by = l / gridDim.x;
  }
  const int seq = items[2 * bx], qb = items[2 * bx + 1];
  const int NHG = G / HPW;
  const int kvh = by / NHG, hg = by % NHG;
  const int TPW = 4 / HPW;
  const int qs = q_start[seq], ql = q_len[seq], ctx = ctx_len[seq];
  const int pbase = ctx - ql;
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const int head = kvh * G + hg * HPW + (w % HPW);
  const int tok0 = qb + (w / HPW) * 32;
  const int ntok = max(0, min(32, ql - tok0));
  const int p_lo = pbase + tok0, p_hi = pbase + tok0 + max(ntok, 1) - 1;
  const int wg_tok_end = min(ql, qb + 32 * TPW);
  const int wg_p_lo = pbase + qb, wg_p_hi = pbase + wg_tok_end - 1;
  const int kmin = window > 0 ? max(0, wg_p_lo - window + 1) : 0;
  const int t_first = kmin >> 6, t_last = wg_p_hi >> 6;

  // Q^T fragments (B operand): lane l holds Q[tok0 + l32][16 ks + 8 h + j]
  bf16x8_t qf[8];
  {
    const int tk = tok0 + l32;
    const uint16_t* qr = q + (int64_t)(qs + min(tk, ql - 1)) * q_stride + (int64_t)head * D;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      u32x4_t v = {0, 0, 0, 0};
      if (tk < ql) v = *reinterpret_cast<const u32x4_t*>(qr + (2 * ks + h) * 8);
      qf[ks] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  const int qp = p_lo + l32;  // this lane's query position
  float m = NEG_INF, lsum = 0.f;
  f32x16_t o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f32x16_t{};

  // DMA (v2's): wave w issues 1-KB pieces j = w + 4 i of K and V; lane -> row u / 16, slot u % 16
  const int ws = __builtin_amdgcn_readfirstlane(w);
  uint32_t koff[NI / 4];
#pragma unroll
  for (int i = 0; i < NI / 4; ++i) {
    const int u = 64 * (w + 4 * i) + lane;
    const int row = u / 16, sl = u % 16;
    koff[i] = (uint32_t)(row * RB + 16 * (sl ^ p4_sw(row)));
  }
  auto dma = [&](const char* src, char* dst) {
    // V4 bit 1: the DMA from asm (glds16), so hipcc's waitcnt pass keeps counting LDS reads
    // (a visible global_load_lds in the loop turns every fragment wait into lgkmcnt(0))
    if constexpr (V4 & 2) glds16(src, lds_addr(dst));
    else __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                          (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  auto issue = [&](char* base, int t) {
    const int ts = t * 64;
    LLMD_DCHECK(ts < ctx && bt[ts >> lbs] >= 0 && ctx <= bt_stride * bs);
    const int64_t tb = 2 * ((int64_t)bt[ts >> lbs] * block_stride + head_off + (int64_t)(ts & (bs - 1)) * D);
    const char* kb = reinterpret_cast<const char*>(kc) + tb;
    const char* vb = reinterpret_cast<const char*>(vc) + tb;
    const int rlim = ctx - 1 - ts;
    if (rlim >= 63 && bs >= 64) {
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        char* dst = base + 1024 * (ws + 4 * i);
        dma(kb + koff[i], dst);
        dma(vb + koff[i], dst + IMG);
      }
    } else if (rlim >= 63) {
      // blocks of 16 / 32 keys: a piece's 4 rows sit in one block
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        const int r0 = 4 * (ws + 4 * i);
        const int key0 = ts + r0;
        const int64_t ib = 2 * ((int64_t)bt[key0 >> lbs] * block_stride + head_off + (int64_t)(key0 & (bs - 1)) * D) -
                           (int64_t)r0 * RB;
        char* dst = base + 1024 * (ws + 4 * i);
        dma(reinterpret_cast<const char*>(kc) + ib + koff[i], dst);
        dma(reinterpret_cast<const char*>(vc) + ib + koff[i], dst + IMG);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI / 4; ++i) {
        const int u = 64 * (w + 4 * i) + lane;
        const int row = u / 16, sl = u % 16;
        const int key = ts + min(row, rlim);  // rows past the end re-read the last key (finite V, P = 0)
        const int64_t ro = bs >= 64 ? (int64_t)min(row, rlim) * RB
                                    : 2 * ((int64_t)bt[key >> lbs] * block_stride + head_off +
                                           (int64_t)(key & (bs - 1)) * D) - tb;
        char* dst = base + 1024 * (ws + 4 * i);
        dma(kb + ro + 16 * (sl ^ p4_sw(row)), dst);
        dma(vb + ro + 16 * (sl ^ p4_sw(row)), dst + IMG);
      }
    }
  };
  // K (A operand) row reads: row 32 kb + l32, chunk 2 ks + h; the swizzle depends on l32 & 15 only
  const int swk = p4_sw(l32);
  int kofs[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) kofs[ks] = l32 * RB + 16 * ((2 * ks + h) ^ swk);
  // V^T (A operand) transposed reads: 16-lane group gr = lane >> 4 (column half gr & 1, key half h),
  // lane 4 qq + pp supplies row r0 + qq, columns 32 db + 16 (gr & 1) + 4 pp .. + 3; two reads per
  // fragment at key rows 4 h + qq and 8 + 4 h + qq (+ 16 s + 32 kb: multiples of 16, same swizzle)
  const int qq = (lane & 15) >> 2, pp = lane & 3, gc = (lane >> 4) & 1;
  int vofs[4][2];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int r = 8 * hh + 4 * h + qq, ch = 4 * db + 2 * gc + (pp >> 1);
      vofs[db][hh] = IMG + r * RB + 16 * (ch ^ p4_sw(r)) + 8 * (pp & 1);
    }

  auto compute = [&](const char* img, int t) {
    const int ts = t * 64;
    const bool active = ntok > 0 && ts <= p_hi && (window <= 0 || ts + 63 > p_lo - window);
    if (!active) return;
    constexpr int PF = 4;
    auto kread = [&](int j) {  // fragment j = 8 kb + ks
      return *reinterpret_cast<const bf16x8_t*>(img + kofs[j % 8] + (j / 8) * 32 * RB);
    };
    auto vread = [&](int j) {  // fragment j = 4 db + ks2 (keys 16 ks2 ..)
      const char* p0 = img + vofs[j / 4][0] + 16 * (j % 4) * RB;
      const char* p1 = img + vofs[j / 4][1] + 16 * (j % 4) * RB;
      s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
      s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p1);
      return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    };
    f32x16_t sc[2];
    bf16x8_t kr[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) kr[j] = kread(j);
    if constexpr (V4 & 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16_t a;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int j = 8 * kb + ks;
        const bf16x8_t ka = kr[j % PF];
        if (j + PF < 16) kr[j % PF] = kread(j + PF);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], ks == 0 ? f32x16_t{} : a, 0, 0, 0);
        if constexpr (V4 & 1) __builtin_amdgcn_sched_barrier(0);
      }
      sc[kb] = a;
    }
    bf16x8_t vr[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) vr[j] = vread(j);
    const bool need_mask = (ts + 63 > p_lo) || (window > 0 && ts <= p_hi - window);
    if (need_mask) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = ts + 32 * kb + (r & 3) + 8 * (r >> 2) + 4 * h;
          bool ok = key <= qp;
          if (window > 0) ok = ok && key > qp - window;
          sc[kb][r] = ok ? sc[kb][r] : NEG_INF;
        }
    }
    float mx = NEG_INF;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kb][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const float mt = mx * scale_log2;
    if (__ballot(mt > m + 8.f) != 0) {  // lazy rescale (v2's threshold), wave-uniform branch
      const float mnew = fmaxf(m, mt);
      const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
      lsum *= alpha;
      m = mnew;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
    const float msub = (m == NEG_INF) ? 0.f : m;
    float ps = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], scale_log2, -msub));
        sc[kb][r] = p;
        ps += p;
      }
    lsum += ps;  // lane-partial (this half's keys): the halves are summed once, in the epilogue
    bf16x8_t pb[4];  // P^T fragments of key steps 2 kb + s2: registers 8 s2 .. 8 s2 + 7 of sc[kb]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[2 * kb + s2][j] = (__bf16)sc[kb][8 * s2 + j];
    if constexpr (V4 & 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int db = j / 4, ks2 = j % 4;
      const bf16x8_t va = vr[j % PF];
      if (j + PF < 16) vr[j % PF] = vread(j + PF);
      o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb[ks2], o[db], 0, 0, 0);
      if constexpr (V4 & 1) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // V4 bit 2: the two 32-key halves of a tile software-pipelined inside the wave - the MFMAs of
  // S^T half 1 run beside the mask / max VALU of half 0, and the PV MFMAs of half 0 beside the exp /
  // cvt VALU of half 1 (sched_group_barrier interleave: one MFMA, then its share of VALU and LDS
  // reads), so the softmax no longer sits serially between the two products.
  auto compute_p = [&](const char* img, int t) {
    const int ts = t * 64;
    const bool active = ntok > 0 && ts <= p_hi && (window <= 0 || ts + 63 > p_lo - window);
    if (!active) return;
    auto kread = [&](int kb, int ks) {
      return *reinterpret_cast<const bf16x8_t*>(img + kofs[ks] + kb * 32 * RB);
    };
    auto vread = [&](int db, int ks2) {
      const char* p0 = img + vofs[db][0] + 16 * ks2 * RB;
      const char* p1 = img + vofs[db][1] + 16 * ks2 * RB;
      s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
      s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p1);
      return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    };
    const bool need_mask = (ts + 63 > p_lo) || (window > 0 && ts <= p_hi - window);
    auto mask = [&](f32x16_t& x, int kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = ts + 32 * kb + (r & 3) + 8 * (r >> 2) + 4 * h;
        bool ok = key <= qp;
        if (window > 0) ok = ok && key > qp - window;
        x[r] = ok ? x[r] : NEG_INF;
      }
    };
    // S^T half 0, with the half-1 K fragments read beside it
    bf16x8_t k0[8], k1[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) k0[ks] = kread(0, ks);
    f32x16_t s0, s1;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0[ks], qf[ks], ks == 0 ? f32x16_t{} : s0, 0, 0, 0);
      k1[ks] = kread(1, ks);
    }
    if (need_mask) mask(s0, 0);
    // region A: S^T half 1 beside the max of half 0 and the half-0 V fragment reads
    bf16x8_t v0[8];
    float mx = NEG_INF;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1[ks], qf[ks], ks == 0 ? f32x16_t{} : s1, 0, 0, 0);
      mx = fmaxf(mx, fmaxf(s0[2 * ks], s0[2 * ks + 1]));
      v0[ks] = vread(ks >> 1, ks & 1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // VALU
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
    }
    if (need_mask) mask(s1, 1);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s1[r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const float mt = mx * scale_log2;
    if (__ballot(mt > m + 8.f) != 0) {
      const float mnew = fmaxf(m, mt);
      const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
      lsum *= alpha;
      m = mnew;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;
    }
    const float msub = (m == NEG_INF) ? 0.f : m;
    float ps = 0.f;
    bf16x8_t p0[2], p1[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(fmaf(s0[r], scale_log2, -msub));
      ps += p;
      p0[r >> 3][r & 7] = (__bf16)p;
    }
    // region B: PV half 0 beside the exp / cvt of half 1 and the half-1 V fragment reads
    bf16x8_t v1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int db = j >> 1, s2 = j & 1;
      o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0[j], p0[s2], o[db], 0, 0, 0);
      v1[j] = vread(db, 2 + s2);
#pragma unroll
      for (int r = 2 * j; r < 2 * j + 2; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s1[r], scale_log2, -msub));
        ps += p;
        p1[r >> 3][r & 7] = (__bf16)p;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 6, 1);  // VALU
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);  // DS read
    }
    lsum += ps;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int db = j >> 1, s2 = j & 1;
      o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1[j], p1[s2], o[db], 0, 0, 0);
    }
  };

  issue(buf0, t_first);
  for (int t = t_first; t <= t_last; t += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 <= t_last) issue(buf1, t + 1);
    if constexpr (V4 & 4) compute_p(buf0, t); else compute(buf0, t);
    if (t + 1 > t_last) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 2 <= t_last) issue(buf0, t + 2);
    if constexpr (V4 & 4) compute_p(buf1, t + 1); else compute(buf1, t + 1);
  }

  if (ntok == 0) return;
  const float sink = sinks ? sinks[head] * 1.4426950408889634f : NEG_INF;
  float den;
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum), __float_as_uint(lsum), false, false);
    den = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  if (sinks) den += exp2f(sink - (m == NEG_INF ? 0.f : m));
  const float inv = den > 0.f ? vscale / den : 0.f;
  const int tk = tok0 + l32;
  if (tk < ql) {
    uint16_t* orow = out + (int64_t)(qs + tk) * out_stride + (int64_t)head * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {  // d = 32 db + 8 g4 + 4 h + (0..3)
        u32x2_t p;
        p[0] = (uint32_t)f2bf(o[db][4 * g4] * inv) | ((uint32_t)f2bf(o[db][4 * g4 + 1] * inv) << 16);
        p[1] = (uint32_t)f2bf(o[db][4 * g4 + 2] * inv) | ((uint32_t)f2bf(o[db][4 * g4 + 3] * inv) << 16);
        *reinterpret_cast<u32x2_t*>(orow + 32 * db + 8 * g4 + 4 * h) = p;
      }
  }
}
}  // namespace

// v3 for D = 128 bf16 caches with blocks of >= 64 keys and whole groups of 4 query
// heads per KV head (LLMD_PREFILL_V3=1 until its GPU numerics have run on the
// driver's box; v2 otherwise); the single source of the item shape
static bool prefill_v3_ok(int Hq, int Hkv, int D, int bs, int fp8) {
  static const bool off = [] {
    const char* e = getenv("LLMD_PREFILL_V3");
    return !(e && e[0] == '1');
  }();
  static const bool v1_only = [] {
    const char* e = getenv("LLMD_PREFILL_V1");
    return e && e[0] == '1';
  }();
  return !off && !v1_only && D == 128 && !fp8 && bs >= 64 && Hkv > 0 && (Hq / Hkv) % 4 == 0;
}



// v4 (32x32x16 MFMAs) for D = 128 bf16 caches: LLMD_PREFILL_V4=1 (off until its GPU A/B); read per
// launch so one process can A/B both (v4 and v2 share the item shape)
static bool prefill_v4_on() {
  const char* e = getenv("LLMD_PREFILL_V4");
  return e && e[0] == '1';
}

namespace {
// The K / V blocks a prefill step reads from an fp8 (e4m3) paged cache, widened exactly into a dense
// bf16 copy (block table entry e -> row e of the copy): the fp8-KV prefill then runs on the bf16 v2
// kernel (k_scale folded into its softmax scale, v_scale into its epilogue, as for the fp8 kernel)
// instead of the VGPR-staged v1 fp8 kernel (~2x its time at ISL 5000). One workgroup per (entry, K|V);
// 10 MB of K+V per 5000-token layer: a few microseconds.
__global__ __launch_bounds__(256) void kv_dequant_gather_kernel(const uint8_t* __restrict__ kc,
                                                                const uint8_t* __restrict__ vc, int64_t block_stride,
                                                                const int* __restrict__ bt, int n_blocks,
                                                                int per_block, uint16_t* __restrict__ kd,
                                                                uint16_t* __restrict__ vd) {
  const int e = blockIdx.x;
  const int b = min(max(bt[e], 0), n_blocks - 1);  // padding entries (never read by the kernel) -> block 0
  const uint8_t* src = (blockIdx.y ? vc : kc) + (int64_t)b * block_stride;
  uint16_t* dst = (blockIdx.y ? vd : kd) + (int64_t)e * per_block;
  for (int i = threadIdx.x * 8; i < per_block; i += 256 * 8)
    *reinterpret_cast<u32x4_t*>(dst + i) = fp8x8_to_bf16x8(*reinterpret_cast<const u32x2_t*>(src + i));
}
}  // namespace

extern "C" int llmd_kv_dequant_gather(const void* kc, const void* vc, int64_t block_stride, const int* bt,
                                      int n_entries, int n_blocks, int per_block, void* kd, void* vd,
                                      hipStream_t st) {
  if (per_block % 8 || block_stride % 8 || n_blocks <= 0) return -1;
  if (n_entries == 0) return 0;
  hipLaunchKernelGGL(kv_dequant_gather_kernel, dim3(n_entries, 2), dim3(256), 0, st, (const uint8_t*)kc,
                     (const uint8_t*)vc, block_stride, bt, n_blocks, per_block, (uint16_t*)kd, (uint16_t*)vd);
  return (int)hipGetLastError();
}

// the software-pipelined v5 (csrc/ops/attn_prefill5.hip): 1 when the shape is not covered
extern "C" int llmd_paged_prefill_v5(const void* q, int64_t q_stride, const void* kc, const void* vc,
                                     int64_t block_stride, int bs, const int* block_tables, int bt_stride,
                                     const int* q_start, const int* q_len, const int* ctx_len, const int* items,
                                     int n_items, int Hq, int Hkv, int D, float scale_log2, int window,
                                     const float* sinks, void* out, int64_t out_stride, float v_scale, int xcd,
                                     hipStream_t st);

static bool prefill_v5_on() {  // LLMD_PREFILL_V5=1 (read per launch: A/B in one process)
  const char* e = getenv("LLMD_PREFILL_V5");
  return e && e[0] == '1';
}

extern "C" int llmd_paged_prefill(const void* q, int64_t q_stride, const void* kc, const void* vc,
                                  int64_t block_stride, int bs, const int* block_tables,
                                  int bt_stride, const int* q_start, const int* q_len,
                                  const int* ctx_len, const int* items, int n_items, int Hq,
                                  int Hkv, int D, float scale, int window, const float* sinks,
                                  void* out, int64_t out_stride, int fp8, float k_scale, float v_scale,
                                  hipStream_t st) {
  if (n_items == 0) return 0;
  const int G = Hq / Hkv;
  const int HPW = (G % 4 == 0) ? 4 : ((G % 2 == 0) ? 2 : 1);  // 4 / HPW must be integral
  const float scale_log2 = scale * k_scale * 1.4426950408889634f;
  dim3 grid(n_items, Hkv * (G / HPW)), blk(NT);
  static bool attr_done = false;
  if (!attr_done) {
    const int l128 = 2 * (64 * (128 * 2 + 16) + 64 * 128 * 2), l64 = 2 * (64 * (64 * 2 + 16) + 64 * 64 * 2);
    (void)hipFuncSetAttribute((const void*)prefill_kernel<128, false>, hipFuncAttributeMaxDynamicSharedMemorySize, l128);
    (void)hipFuncSetAttribute((const void*)prefill_kernel<128, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l128);
    (void)hipFuncSetAttribute((const void*)prefill_kernel<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, l64);
    (void)hipFuncSetAttribute((const void*)prefill_kernel<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, l64);
    attr_done = true;
  }
#define LAUNCH(DD, F8)                                                                                        \
  hipLaunchKernelGGL((prefill_kernel<DD, F8>), grid, blk, (size_t)(2 * (64 * (DD * 2 + 16) + 64 * DD * 2)), st, \
                     (const uint16_t*)q, q_stride, kc, vc, block_stride, bs, block_tables, bt_stride, q_start,   \
                     q_len, ctx_len, items, Hq, Hkv, G, HPW, scale_log2, window, sinks, (uint16_t*)out,        \
                     out_stride, v_scale)
  static const bool v1_only = [] {
    const char* e = getenv("LLMD_PREFILL_V1");
    return e && e[0] == '1';
  }();
  static const bool xcd_map = [] {  // LLMD_PREFILL_XCD=0: plain round-robin dispatch (A/B)
    const char* e = getenv("LLMD_PREFILL_XCD");
    return !(e && e[0] == '0');
  }();
  if (prefill_v3_ok(Hq, Hkv, D, bs, fp8)) {
    const dim3 grid3(n_items, Hkv * (G / 4));
    hipLaunchKernelGGL(prefill_v3_kernel, grid3, blk, 0, st, (const uint16_t*)q, q_stride, (const uint16_t*)kc,
                       (const uint16_t*)vc, block_stride, bs, block_tables, bt_stride, q_start, q_len, ctx_len,
                       items, Hq, Hkv, G, scale_log2, window, sinks, (uint16_t*)out, out_stride, v_scale,
                       xcd_map && (int64_t)n_items * grid3.y >= 1024 ? 1 : 0);
  } else if (!fp8 && !v1_only && prefill_v5_on() &&
             llmd_paged_prefill_v5(q, q_stride, kc, vc, block_stride, bs, block_tables, bt_stride, q_start, q_len,
                                   ctx_len, items, n_items, Hq, Hkv, D, scale_log2, window, sinks, out, out_stride,
                                   v_scale, xcd_map && (int64_t)n_items * (Hkv * (G / 4)) >= 1024 ? 1 : 0,
                                   st) == 0) {
    // launched by v5
  } else if (D == 128 && !fp8 && bs >= 16 && !v1_only && prefill_v4_on()) {
    const char* e4 = getenv("LLMD_PREFILL_V4_VARIANT");  // 1: builtin DMA, 3: asm DMA, 7: asm DMA + pipelined halves
    auto kern4 = (e4 && e4[0] == '1') ? prefill_v4_kernel<1> : (e4 && e4[0] == '7') ? prefill_v4_kernel<7>
                                                                                     : prefill_v4_kernel<3>;
    hipLaunchKernelGGL(kern4, grid, blk, 0, st, (const uint16_t*)q, q_stride, (const uint16_t*)kc,
                       (const uint16_t*)vc, block_stride, bs, block_tables, bt_stride, q_start, q_len, ctx_len,
                       items, Hq, Hkv, G, HPW, scale_log2, window, sinks, (uint16_t*)out, out_stride, v_scale,
                       xcd_map && (int64_t)n_items * grid.y >= 1024 ? 1 : 0);
  } else if ((D == 128 || D == 64) && !fp8 && bs >= 16 && !v1_only) {
    const int pv = [] {  // read per launch (tests and A/Bs switch it in one process; getenv is ~0.1 us)
      // A/B of the round-4 schedule (V above; profiles/attn_prefill_r4_ab.txt): the ring wins everywhere,
      // the asm DMA only at full ISL and loses 12 % on one-wave grids (5000 x 512 chunk); reading
      // 6 fragments ahead (bit 2) adds ~1 % -> 5
      // round 6 (profiles/attn_prefill_v2_variants_r6.txt): unpacked row sums + buffer-descriptor DMA
      // (bits 4, 5) +1 to +4 % at ISL 2048-8192 -> 53
      // round 6 (r6w): + Q pre-scaled / accumulators started at -m and row sums on the MFMA (bits 7, 8)
      // +3 to +6 % more at D = 128, +7 to +9 % over the round-5 V5 at D = 64 (gpt-oss) -> 437 for both
      const char* e = getenv("LLMD_PREFILL_V2_VARIANT");
      return e ? (atoi(e) & 511) : -1;
    }();
    auto pick = [](int v, bool d128) {  // instantiated: 0-3, 5 (PF 6), 9 (early V), 13 (both); D 128: 21, 37, 53, 69, 117, 181, 309, 437
      if (d128) return v == 0 ? prefill_v2_kernel<128, 0> : v == 2 ? prefill_v2_kernel<128, 2>
                     : v == 3 ? prefill_v2_kernel<128, 3> : v == 5 ? prefill_v2_kernel<128, 5>
                     : v == 9 ? prefill_v2_kernel<128, 9> : v == 13 ? prefill_v2_kernel<128, 13>
                     : v == 21 ? prefill_v2_kernel<128, 21> : v == 37 ? prefill_v2_kernel<128, 37>
                     : v == 53 ? prefill_v2_kernel<128, 53> : v == 69 ? prefill_v2_kernel<128, 69>
                     : v == 117 ? prefill_v2_kernel<128, 117> : v == 181 ? prefill_v2_kernel<128, 181>
                     : v == 309 ? prefill_v2_kernel<128, 309> : v == 437 ? prefill_v2_kernel<128, 437>
                     : prefill_v2_kernel<128, 1>;
      return v == 0 ? prefill_v2_kernel<64, 0> : v == 2 ? prefill_v2_kernel<64, 2>
             : v == 3 ? prefill_v2_kernel<64, 3> : v == 5 ? prefill_v2_kernel<64, 5>
             : v == 9 ? prefill_v2_kernel<64, 9> : v == 13 ? prefill_v2_kernel<64, 13>
             : v == 53 ? prefill_v2_kernel<64, 53> : v == 181 ? prefill_v2_kernel<64, 181>
             : v == 437 ? prefill_v2_kernel<64, 437>
             : prefill_v2_kernel<64, 1>;
    };
    auto kern = pick(pv >= 0 ? pv : 437, D == 128);
    hipLaunchKernelGGL(kern, grid, blk, 0, st, (const uint16_t*)q, q_stride, (const uint16_t*)kc,
                       (const uint16_t*)vc, block_stride, bs, block_tables, bt_stride, q_start, q_len, ctx_len,
                       items, Hq, Hkv, G, HPW, scale_log2, window, sinks, (uint16_t*)out, out_stride, v_scale,
                       xcd_map && (int64_t)n_items * grid.y >= 1024 ? 1 : 0);
  } else if (D == 128) {
    if (fp8) LAUNCH(128, true); else LAUNCH(128, false);
  } else if (D == 64) {
    if (fp8) LAUNCH(64, true); else LAUNCH(64, false);
  } else {
    return -1;
  }
#undef LAUNCH
  return 0;
}

// tokens per work item (host helper, mirrors the kernel llmd_paged_prefill
// dispatches: v3 64; v1 / v2 32 query tokens per wave, 4 / HPW waves stacked
// along the tokens)
extern "C" int llmd_prefill_tokens_per_item(int Hq, int Hkv, int D, int bs, int fp8) {
  if (prefill_v3_ok(Hq, Hkv, D, bs, fp8)) return 64;  // v3: 64 tokens x 4 heads per workgroup
  const int G = Hq / Hkv;
  const int HPW = (G % 4 == 0) ? 4 : ((G % 2 == 0) ? 2 : 1);
  return 32 * (4 / HPW);
}
