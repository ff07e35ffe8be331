// GQA prefill attention v5: attn_prefill.hip's v2 work decomposition and tile
// images (4-wave workgroup = 4 query heads of one GQA group x 32 query tokens, 64-key tiles
// staged in LDS by the DMA and shared by the 4 waves, S^T = K . Q^T so P lands lane-local in the
// PV A-operand layout, V read with ds_read_b64_tr_b16), with the two products of CONSECUTIVE
// tiles software-pipelined inside each wave:
//
//   phase A of step t:  S(t+1) = K(t+1) . Q^T  (32 MFMAs)   ||  P(t) = exp2(S(t) - m), row sums,
//                                                              bf16 packing of P(t)
//   phase B of step t:  O += P(t) . V(t)       (32 MFMAs)   ||  row max of S(t+1) (+ its causal
//                                                              mask on a diagonal tile)
//
// so every VALU instruction of the softmax sits beside an MFMA of the other product instead of
// waiting on its own tile's MFMA chain (v2: QK MFMAs -> max -> exp -> PV MFMAs in one dependency
// chain per tile; only the second wave on the SIMD fills the gaps). Fragments are read a ring of
// PF steps ahead and one sched_barrier closes every step (hipcc's own schedule hoists the reads and
// waits lgkmcnt(0)); the interleave is written out in source order.
//
// K and V live in separate two-slot rings (same 64 KB as v2): at the start of step t (one
// vmcnt(0) + barrier) K(t+1) and V(t) have landed, K(t)'s slot takes K(t+2) and V(t-1)'s slot
// takes V(t+1) - each DMA has a full step to land. The lazy online-softmax rescale (only when a
// row max grows by more than 8 in log2 units) runs after phase B, where O holds P(t) . V(t).
//
// Scope: bf16 cache, D = 128, whole GQA groups of 4 (every wave of a workgroup has the same
// causal range), blocks of >= 64 keys, no sliding window (sinks supported). Other shapes stay on
// v2. Host entry llmd_paged_prefill_v5, dispatched from llmd_paged_prefill (attn_prefill.hip).
#include <type_traits>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int P5_NT = 256;
constexpr float P5_NEG_INF = -__builtin_huge_valf();

__device__ __forceinline__ int p5_rowoff(int g) { return 4 * (g >> 1) + 8 * (g & 1); }
// v2's D = 128 swizzles (attn_prefill.hip p2_pk / p2_pv)
__device__ __forceinline__ int p5_pk(int r) { return ((r >> 1) & 7) | ((r & 1) << 3); }
__device__ __forceinline__ int p5_pv(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

typedef int p5_i32x4 __attribute__((ext_vector_type(4)));

// LDS-DMA of one 1 KB piece through a scalar buffer descriptor, issued from asm: hipcc's waitcnt pass
// does not see the LDS write, so it neither forces vmcnt(0) before the fragment reads of the other ring
// slot nor stops counting lgkmcnt (the kernel orders the DMA itself: vmcnt(0) + barrier per step)
__device__ __forceinline__ void p5_bdma(p5_i32x4 rsrc, uint32_t voff, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

__global__ __launch_bounds__(P5_NT, 2) void prefill_v5_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, int64_t block_stride, int bs, const int* __restrict__ block_tables,
    int bt_stride, const int* __restrict__ q_start, const int* __restrict__ q_len, const int* __restrict__ ctx_len,
    const int* __restrict__ items, int Hq, int Hkv, int G, float scale_log2, const float* __restrict__ sinks,
    uint16_t* __restrict__ out, int64_t out_stride, float vscale, int xcd) {
  constexpr int D = 128, KS = 4, NB = 8, RB = 256;
  constexpr int IMG = 64 * RB;  // one 64-key bf16 image (16 KB)
  constexpr int PF = 4;         // fragments read ahead
  __shared__ __attribute__((aligned(1024))) char lds[4 * IMG];  // K0 | K1 | V0 | V1 (the ONLY LDS object)

  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int l = xcd_remap(by * gridDim.x + bx, gridDim.x * gridDim.y);
    bx = l % gridDim.x;
    by = l / gridDim.x;
  }
  const int seq = items[2 * bx], qb = items[2 * bx + 1];
  const int NHG = G / 4;
  const int kvh = by / NHG, hg = by % NHG;
  const int qs = q_start[seq], ql = q_len[seq], ctx = ctx_len[seq];
  const int pbase = ctx - ql;
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_off = (int64_t)kvh * bs * D;
  const int lbs = __builtin_ctz(bs);

  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int head = kvh * G + hg * 4 + w;
  const int tok0 = qb;  // all 4 waves: the same 32 tokens (4 heads)
  const int p_lo = pbase + tok0;
  const int p_hi = pbase + min(ql, tok0 + 32) - 1;
  const int t_first = 0, t_last = p_hi >> 6;

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
  float m[2] = {P5_NEG_INF, P5_NEG_INF}, lsum[2] = {0.f, 0.f};
  f32x4_t o[2][NB];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int n = 0; n < NB; ++n) o[nb][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // DMA: 16 K + 16 V wave-instructions of 1 KB (4 rows) per tile; wave w issues pieces w + 4 i
  const int ws = __builtin_amdgcn_readfirstlane(w);
  // per-lane source offsets inside a tile, K | V << 16 (both < 16 KB): rows 4 (w + 4 i) + lane / 16,
  // LDS slot lane % 16 <- chunk slot ^ swizzle(row)
  uint32_t kvoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = 64 * (w + 4 * i) + lane;
    const int row = u / (D / 8), sl = u % (D / 8);
    kvoff[i] = (uint32_t)(row * RB + 16 * (sl ^ p5_pk(row))) | ((uint32_t)(row * RB + 16 * (sl ^ p5_pv(row))) << 16);
  }
  auto issue = [&](const uint16_t* cache, int t, bool is_v) {
    char* base = lds + (is_v ? 2 * IMG : 0) + (t & 1) * IMG;
    const int ts = t * 64;
    const int64_t tb = 2 * ((int64_t)bt[ts >> lbs] * block_stride + head_off + (int64_t)(ts & (bs - 1)) * D);
    const uint64_t src = (uint64_t)(uintptr_t)cache + (uint64_t)tb;
    // rows past the sequence's end (its last, partial tile) read zeros through the descriptor's range:
    // finite V rows (P = 0 there; 0 * NaN would poison O)
    const int rows = min(64, ctx - ts);
    p5_i32x4 rsrc;
    rsrc[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)src);
    rsrc[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(src >> 32) & 0xffffu));
    rsrc[2] = __builtin_amdgcn_readfirstlane(rows * RB);
    rsrc[3] = 0x00020000;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      p5_bdma(rsrc, is_v ? (kvoff[i] >> 16) : (kvoff[i] & 0xffffu), lds_addr(base + 1024 * (ws + 4 * i)));
  };
  const int qq = c16 >> 2, pp = c16 & 3;
  const int srow = p5_rowoff(c16 >> 2) + (c16 & 3), kp = p5_pk(srow);
  int kofs[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) kofs[s] = srow * RB + 16 * ((4 * s + g) ^ kp);
  const int vrow = p5_rowoff(g) + qq, vp = p5_pv(vrow);
  int vofs[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) vofs[n] = vrow * RB + 16 * ((2 * n + (pp >> 1)) ^ vp) + 8 * (pp & 1);
  auto kread = [&](const char* img, int j) {
    return *reinterpret_cast<const bf16x8_t*>(img + kofs[j % KS] + (j / KS) * 16 * RB);
  };
  auto vread = [&](const char* img, int j) {
    const char* p0 = img + vofs[j % NB] + 32 * (j / NB) * RB;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * RB));
    return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
  };

  // S tiles: sc[b4][nb][i] = S[key ts + 16 b4 + rowoff(g) + i][query 16 nb + c16]
  f32x4_t sc[4][2], sn[4][2];
  // the causal mask of tile t on S (diagonal tiles only: keys past the wave's first query)
  auto mask = [&](f32x4_t (&s)[4][2], int t) {
    const int ts = t * 64;
    if (ts + 63 > p_lo) {  // wave-uniform
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int qp = p_lo + 16 * nb + c16;
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = ts + 16 * b4 + p5_rowoff(g) + i;
            s[b4][nb][i] = key <= qp ? s[b4][nb][i] : P5_NEG_INF;
          }
      }
    }
  };
  // the lazy rescale: the new row maxima of tile S (lane-partial maxima mt) and, when one grows by
  // more than 8, O / lsum rescaled (cross-lane reductions only then)
  auto rescale = [&](const float (&mt)[2]) {
    bool grow = false;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) grow = grow || (mt[nb] > m[nb] + 8.f);
    if (__ballot(grow) != 0) {
      float alpha[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        float mx = fmaxf(mt[nb], __shfl_xor(mt[nb], 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[nb], mx);
        alpha[nb] = (mnew == P5_NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m[nb] - mnew);
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
  };

  // ---- prologue: K(0), V(0), K(1); S(0), its mask and maxima
  issue(kc, t_first, false);
  issue(vc, t_first, true);
  if (t_first + 1 <= t_last) issue(kc, t_first + 1, false);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  {
    const char* img = lds + (t_first & 1) * IMG;
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8_t ka = kread(img, KS * b4 + s);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[0][s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[1][s], a1, 0, 0, 0);
      }
      sc[b4][0] = a0;
      sc[b4][1] = a1;
    }
    mask(sc, t_first);
    float mt[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float mx = P5_NEG_INF;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) mx = fmaxf(mx, fmaxf(fmaxf(sc[b4][nb][0], sc[b4][nb][1]), fmaxf(sc[b4][nb][2], sc[b4][nb][3])));
      mt[nb] = mx * scale_log2;
    }
    rescale(mt);
  }

  // softmax element e of the current tile (e = 16 nb + 4 b4 + i): p = 2^(S scale - m), row sum
  float ps[2];
  auto sm_elem = [&](int e) {
    const int nb = e >> 4, b4 = (e >> 2) & 3, i = e & 3;
    const float msub = (m[nb] == P5_NEG_INF) ? 0.f : m[nb];
    const float p = __builtin_amdgcn_exp2f(fmaf(sc[b4][nb][i], scale_log2, -msub));
    sc[b4][nb][i] = p;
    ps[nb] += p;
    asm volatile("" : "+v"(ps[nb]));  // scalar adds (no v_pk_add_f32 beside the MFMAs)
  };
  bf16x8_t pa[2][2];
  auto pack = [&](int t2, int nb) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pa[t2][nb][j] = (__bf16)sc[2 * t2][nb][j];
      pa[t2][nb][4 + j] = (__bf16)sc[2 * t2 + 1][nb][j];
    }
    asm volatile("" : "+v"(pa[t2][nb]));  // converted here, beside phase A's MFMAs (not sunk past the mask)
  };

  // one pipelined step; MORE: a next tile exists (the last step has no S(t+1) to overlap)
  auto step = [&](auto more_, int t) {
    constexpr bool more = decltype(more_)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K(t+1), V(t) landed
    __syncthreads();                                   // K(t) and V(t-1) slots free in every wave
    if (t + 2 <= t_last) issue(kc, t + 2, false);
    if constexpr (more) issue(vc, t + 1, true);
    const char* kimg = lds + ((t + 1) & 1) * IMG;
    const char* vimg = lds + 2 * IMG + (t & 1) * IMG;
    ps[0] = ps[1] = 0.f;
    if constexpr (more) {
      // ---- phase A: S(t+1) MFMAs || softmax of S(t)
      bf16x8_t kr[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) kr[j] = kread(kimg, j);
      __builtin_amdgcn_sched_barrier(0);
      f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4 * KS; ++j) {
        const int b4 = j / KS, s = j % KS;
        const bf16x8_t ka = kr[j % PF];
        if (j + PF < 4 * KS) kr[j % PF] = kread(kimg, j + PF);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[0][s], a0, 0, 0, 0);
        sm_elem(2 * j);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[1][s], a1, 0, 0, 0);
        sm_elem(2 * j + 1);
        if (s == KS - 1) {
          sn[b4][0] = a0;
          sn[b4][1] = a1;
          a0 = f32x4_t{0.f, 0.f, 0.f, 0.f};
          a1 = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
        if (j == 3) pack(0, 0);   // elements 0..7: b4 0, 1 of nb 0
        if (j == 7) pack(1, 0);
        if (j == 11) pack(0, 1);
        if (j == 15) pack(1, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 32; ++e) sm_elem(e);
      pack(0, 0);
      pack(1, 0);
      pack(0, 1);
      pack(1, 1);
    }
    lsum[0] += ps[0];
    lsum[1] += ps[1];
    // ---- phase B: O += P(t) . V(t) || mask + row maxima of S(t+1)
    if constexpr (more) mask(sn, t + 1);
    float mx[2] = {P5_NEG_INF, P5_NEG_INF};
    {
      bf16x8_t vr[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) vr[j] = vread(vimg, j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2 * NB; ++j) {
        const int t2 = j / NB, n = j % NB;
        const bf16x8_t vb = vr[j % PF];
        if (j + PF < 2 * NB) vr[j % PF] = vread(vimg, j + PF);
        o[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[t2][0], vb, o[0][n], 0, 0, 0);
        o[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[t2][1], vb, o[1][n], 0, 0, 0);
        if (more && j < 8) {  // (nb, b4) = (j / 4, j % 4): one max pair per step (compile-time)
          const int nb = j >> 2, b4 = j & 3;
          mx[nb] = fmaxf(mx[nb], fmaxf(fmaxf(sn[b4][nb][0], sn[b4][nb][1]), fmaxf(sn[b4][nb][2], sn[b4][nb][3])));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (more) {
      const float mt[2] = {mx[0] * scale_log2, mx[1] * scale_log2};
      rescale(mt);  // O now holds P(t) . V(t): rescaling it to S(t+1)'s maxima is exact
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) {
        sc[b4][0] = sn[b4][0];
        sc[b4][1] = sn[b4][1];
      }
    }
  };
  for (int t = t_first; t < t_last; ++t) step(std::integral_constant<bool, true>{}, t);
  step(std::integral_constant<bool, false>{}, t_last);

  const float sink = sinks ? sinks[head] * 1.4426950408889634f : P5_NEG_INF;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    float den = lsum[nb] + __shfl_xor(lsum[nb], 16, 64);
    den += __shfl_xor(den, 32, 64);
    if (sinks) den += exp2f(sink - (m[nb] == P5_NEG_INF ? 0.f : m[nb]));
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

}  // namespace

// v5 for bf16 caches with D = 128, Hq / Hkv % 4 == 0, blocks of >= 64 keys, no sliding window;
// the items are v2's (32 query tokens each). Returns 1 when the shape is not covered (caller
// falls back to v2), 0 on launch.
extern "C" int llmd_paged_prefill_v5(const void* q, int64_t q_stride, const void* kc, const void* vc,
                                     int64_t block_stride, int bs, const int* block_tables, int bt_stride,
                                     const int* q_start, const int* q_len, const int* ctx_len, const int* items,
                                     int n_items, int Hq, int Hkv, int D, float scale_log2, int window,
                                     const float* sinks, void* out, int64_t out_stride, float v_scale, int xcd,
                                     hipStream_t st) {
  const int G = Hq / Hkv;
  if (D != 128 || G % 4 != 0 || bs < 64 || (bs & (bs - 1)) || window > 0) return 1;
  if (n_items == 0) return 0;
  const dim3 grid(n_items, Hkv * (G / 4));
  hipLaunchKernelGGL(prefill_v5_kernel, grid, dim3(P5_NT), 0, st, (const uint16_t*)q, q_stride, (const uint16_t*)kc,
                     (const uint16_t*)vc, block_stride, bs, block_tables, bt_stride, q_start, q_len, ctx_len, items, Hq,
                     Hkv, G, scale_log2, sinks, (uint16_t*)out, out_stride, v_scale, xcd);
  return 0;
}
