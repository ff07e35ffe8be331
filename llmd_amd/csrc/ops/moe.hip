// Mixture-of-Experts kernels: gating top-k, expert
// alignment/permutation, MFMA grouped GEMM with fused epilogues, combine.
//
//   moe_topk      one wave per token: softmax / sigmoid scoring, optional
//                 per-expert bias (DeepSeek correction bias), grouped top-k
//                 (n_group / topk_group), renormalisation, routed scaling.
//   moe_align     per-expert counts -> offsets padded to the GEMM M-tile ->
//                 sorted_ids[P] (token*topk + slot, -1 for padding) and the
//                 expert id of every M-tile; single workgroup (T*k <= 64k).
//   moe_gemm      grouped GEMM  Y[p, :] = X[tok(p), :] . W[e(tile)]^T
//                 MFMA 16x16x32 bf16, 64x128 output tile per 256-thread
//                 workgroup (2x2 waves of 32x64), K-step 64 double-buffered
//                 in LDS with register staging (next tile's loads in flight
//                 during the current tile's MFMAs). A rows are gathered by
//                 sorted_ids; W is [E, N, K] row-major so both operands are
//                 K-contiguous rows (16-B loads, ds_read_b128 fragments).
//                 Epilogue modes: 0 = store bf16, 1 = gated act on an
//                 interleaved [g0,u0,g1,u1..] N axis (SiLU or gpt-oss clamped
//                 SwiGLU) storing N/2 columns.
//   moe_combine   out[t] = sum_j w[t,j] * Y[inv(t,j)]  (deterministic, no atomics)
// Weights of every expert are read exactly once per M-tile, which at decode
// sizes (a few tokens per expert) is the HBM-bound optimum.
#include <cstdlib>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr float NEG_INF = -__builtin_huge_valf();

// ---------------------------------------------------------------- gating
// scoring: 0 softmax over all experts, 1 sigmoid, 2 softmax over the selected top-k (gpt-oss)
__global__ __launch_bounds__(256) void moe_topk_kernel(const float* __restrict__ logits, int T, int E, int K,
                                                       int scoring, const float* __restrict__ bias,
                                                       int n_group, int topk_group, int renorm,
                                                       float routed_scale, int* __restrict__ ids,
                                                       float* __restrict__ wts) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + wave;
  if (t >= T) return;
  const float* l = logits + (int64_t)t * E;
  constexpr int MAXV = 8;  // up to 512 experts
  float sc[MAXV], sel[MAXV];
  const int nv = (E + 63) / 64;
  float mx = NEG_INF;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = lane + 64 * i;
    float v = (i < nv && e < E) ? l[e] : NEG_INF;
    sc[i] = v;
    mx = fmaxf(mx, v);
  }
  if (scoring == 0) {
    mx = wave_max(mx);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      sc[i] = (sc[i] == NEG_INF) ? 0.f : __expf(sc[i] - mx);
      s += sc[i];
    }
    s = wave_sum(s);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) sc[i] /= s;
  } else if (scoring == 1) {
#pragma unroll
    for (int i = 0; i < MAXV; ++i) sc[i] = (sc[i] == NEG_INF) ? 0.f : 1.f / (1.f + __expf(-sc[i]));
  }
  // selection scores (+ bias); invalid experts -inf
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = lane + 64 * i;
    sel[i] = (i < nv && e < E) ? sc[i] + (bias ? bias[e] : 0.f) : NEG_INF;
  }
  // group-limited routing: keep topk_group groups by the sum of their top-2 selection scores
  if (n_group > 1) {
    const int gsz = E / n_group;
    __shared__ float gscore[4][64];
    __shared__ int gkeep[4][64];
    if (lane < n_group) {
      float a = NEG_INF, b = NEG_INF;
      for (int j = 0; j < gsz; ++j) {
        const int e = lane * gsz + j;
        float v = l[e];
        if (scoring == 1) v = 1.f / (1.f + __expf(-v));
        else if (scoring == 0) v = __expf(v - mx);
        v += bias ? bias[e] : 0.f;
        if (v > a) { b = a; a = v; } else if (v > b) b = v;
      }
      gscore[wave][lane] = a + (gsz > 1 ? b : 0.f);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      for (int g = 0; g < n_group; ++g) gkeep[wave][g] = 0;
      for (int r = 0; r < topk_group; ++r) {
        int best = -1;
        float bv = NEG_INF;
        for (int g = 0; g < n_group; ++g)
          if (!gkeep[wave][g] && gscore[wave][g] > bv) { bv = gscore[wave][g]; best = g; }
        if (best >= 0) gkeep[wave][best] = 1;
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int e = lane + 64 * i;
      if (e < E && !gkeep[wave][e / gsz]) sel[i] = NEG_INF;
    }
  }
  // iterative top-k by wave argmax
  float wsum = 0.f, myw = 0.f;
  int myid = 0;
  float topv[16];
  for (int k = 0; k < K; ++k) {
    float bv = NEG_INF;
    int bi = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int e = lane + 64 * i;
      if (sel[i] > bv || (sel[i] == bv && e < bi)) { bv = sel[i]; bi = e; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    // gate weight: the unbiased score of the chosen expert
    float w = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int e = lane + 64 * i;
      if (e == bi) {
        w = (scoring == 2) ? l[e] : sc[i];
        sel[i] = NEG_INF;
      }
    }
    w = wave_sum(w);  // exactly one lane contributed
    if (k < 16) topv[k] = w;
    if (lane == k) { myid = bi; myw = w; }
  }
  if (scoring == 2) {  // softmax over the selected logits
    float m2 = NEG_INF;
    for (int k = 0; k < K && k < 16; ++k) m2 = fmaxf(m2, topv[k]);
    float s = 0.f;
    for (int k = 0; k < K && k < 16; ++k) s += __expf(topv[k] - m2);
    myw = __expf(myw - m2) / s;
  } else if (renorm) {
    for (int k = 0; k < K && k < 16; ++k) wsum += topv[k];
    myw = myw / (wsum > 0.f ? wsum : 1.f);
  }
  if (lane < K) {
    ids[(int64_t)t * K + lane] = myid;
    wts[(int64_t)t * K + lane] = myw * routed_scale;
  }
}

// ---------------------------------------------------------------- align
__global__ __launch_bounds__(1024) void moe_align_kernel(const int* __restrict__ ids, int n, int E, int BM,
                                                         int* __restrict__ sorted_ids, int* __restrict__ tile_expert,
                                                         int* __restrict__ expert_offsets, int max_p,
                                                         int* __restrict__ total_p, int* __restrict__ inv) {
  extern __shared__ int sm[];  // counts[E], offs[E+1], cursor[E]
  int* cnt = sm;
  int* off = sm + E;
  int* cur = sm + 2 * E + 1;
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    if (e >= 0 && e < E) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      off[e] = acc;
      acc += ((cnt[e] + BM - 1) / BM) * BM;
    }
    off[E] = acc;
    *total_p = acc;
  }
  __syncthreads();
  const int P = off[E];
  for (int p = threadIdx.x; p < max_p; p += blockDim.x) sorted_ids[p] = -1;
  for (int i = threadIdx.x; i < n; i += blockDim.x) inv[i] = -1;  // pairs routed off this rank stay -1
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    cur[e] = off[e];
    expert_offsets[e] = off[e];
    for (int tt = off[e] / BM; tt < off[e + 1] / BM; ++tt) tile_expert[tt] = e;
  }
  if (threadIdx.x == 0) expert_offsets[E] = P;
  for (int tt = P / BM + threadIdx.x; tt < max_p / BM; tt += blockDim.x) tile_expert[tt] = -1;
  __syncthreads();
  // parallel scatter through LDS cursors. The order of rows inside an expert
  // segment is not fixed, but every row's GEMM result is independent of its
  // neighbours and moe_combine reads rows through `inv`, so outputs are
  // bitwise identical run to run.
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    if (e >= 0 && e < E) sorted_ids[atomicAdd(&cur[e], 1)] = i;
  }
}

// ---------------------------------------------------------------- grouped GEMM
constexpr int BM = 64, BN = 128, BK = 64, NT = 256;
constexpr int LDA = BK + 8;  // padded LDS row (elements): 144 B rows -> conflict-light b128 reads

template <int MODE>
__global__ __launch_bounds__(NT, 2) void moe_gemm_kernel(
    const uint16_t* __restrict__ X, int64_t x_stride, int topk, const int* __restrict__ sorted_ids,
    const int* __restrict__ tile_expert, const uint16_t* __restrict__ W, int64_t w_expert_stride, int N, int K,
    uint16_t* __restrict__ Y, int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots,
    const uint16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM][LDA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN][LDA];
  const int mt = blockIdx.y, nt = blockIdx.x;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const uint16_t* We = W + (int64_t)e * w_expert_stride;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w >> 1, wn = w & 1;  // wave tile 32 x 64
  // staging: A tile 64 rows x 64 k = 512 chunks (2 per thread); B 128 x 64 = 1024 (4 per thread)
  int arow[2], achk[2];
  const uint16_t* aptr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + NT * i;
    arow[i] = c >> 3;
    achk[i] = c & 7;
    const int sid = sorted_ids[m0 + arow[i]];
    const int tok = sid < 0 ? -1 : (a_rows_are_slots ? m0 + arow[i] : sid / topk);
    aptr[i] = tok < 0 ? nullptr : X + (int64_t)tok * x_stride;
  }
  u32x4_t ra[2], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      u32x4_t v = {0, 0, 0, 0};
      if (aptr[i] && k0 + achk[i] * 8 < K) v = *reinterpret_cast<const u32x4_t*>(aptr[i] + k0 + achk[i] * 8);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      const int r = c >> 3, ch = c & 7;
      u32x4_t v = {0, 0, 0, 0};
      if (n0 + r < N && k0 + ch * 8 < K)
        v = *reinterpret_cast<const u32x4_t*>(We + (int64_t)(n0 + r) * K + k0 + ch * 8);
      rb[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4_t*>(&As[buf][arow[i]][achk[i] * 8]) = ra[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      *reinterpret_cast<u32x4_t*>(&Bs[buf][c >> 3][(c & 7) * 8]) = rb[i];
    }
  };
  f32x4_t acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  const int r16 = lane & 15, kq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[2], bfr[4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(&As[buf][wm * 32 + i * 16 + r16][ks * 32 + kq * 8]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(&Bs[buf][wn * 64 + j * 16 + r16][ks * 32 + kq * 8]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      __syncthreads();
      store(buf ^ 1);
      __syncthreads();
    }
  }
  // epilogue: C[row = 4*kq + r][col = r16] within each 16x16 fragment
  // the expert bias of this lane's columns, loaded once (not once per accumulator element)
  float bvj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + r16;
    bvj[j] = (bias && col < N) ? bf2f(bias[(int64_t)e * N + col]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + i * 16 + kq * 4 + r;
      if (sorted_ids[row] < 0) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + r16;
        float v = acc[i][j][r];
        v += bvj[j];
        if (MODE == 0) {
          if (col < N) Y[(int64_t)row * y_stride + col] = f2bf(v);
        } else {
          // interleaved gate/up: even col = gate, odd col = up (partner lane r16^1)
          const float other = __shfl_xor(v, 1, 64);
          if ((r16 & 1) == 0) {
            float g = v, u = other, o;
            if (act == 2) {
              g = fminf(g, limit);
              u = fminf(fmaxf(u, -limit), limit);
              o = (u + 1.f) * g / (1.f + __expf(-alpha * g));
            } else {
              o = g / (1.f + __expf(-g)) * u;
            }
            if (col < N) Y[(int64_t)row * y_stride + col / 2] = f2bf(o);
          }
        }
      }
    }
  }
}


// ---------------------------------------------------------------- grouped GEMM v2 (LDS-DMA)
// Same contract as moe_gemm_kernel (64-row expert tiles from moe_align), for
// K % 64 == 0. 64 x 256 output tile per 256-thread workgroup, each wave 64 x 64
// (4 x 4 mfma_f32_16x16x32_bf16 tiles, 64 accumulator VGPRs). Operands go
// global -> LDS with global_load_lds_dwordx4 (no VGPR staging, per-lane source
// addresses do the sorted-row gather), two LDS buffers in separate
// allocations so the compiler can see the next tile's DMA does not alias the
// tile being read, one vmcnt(0) + barrier per K-step. LDS rows are 128 B
// (64 bf16) with the 16-B chunk XOR-swizzled by (row >> 1) & 7 on the SOURCE
// side (DMA images are lane-linear): every ds_read_b128 lane group of a
// fragment read then covers 16 distinct slots of a 256-B bank row.
constexpr int G2_BM = 64, G2_BN = 256, G2_NT = 256, G2_MAX_KB = 64;
constexpr int G2_AB = G2_BM * 128, G2_BB = G2_BN * 128, G2_BUF = G2_AB + G2_BB;

__device__ __forceinline__ int g2_swz(int row, int c) { return c ^ ((row >> 1) & 7); }

template <int POL = 0>  // POL 2: nt policy (the expert-weight stream of decode-sized steps)
__device__ __forceinline__ void g2_dma(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds_base, 16, 0, POL);
}
// Expert weights of the v2 kernels (the steps below the v3 row threshold: decode, small mixed
// steps - an expert's panel is read by one or two row tiles) with the nt policy by default
// (LLMD_MOE_NT=0: default policy, for A/B). gpt-oss-120b decode: fp8 batch 256 38.9 -> 36.8 ms,
// bf16 batch 112 44.4 -> 41.7 ms (profiles/decode_nt_r4.txt)
static bool moe_nt() {
  static const bool v = [] {
    const char* e = getenv("LLMD_MOE_NT");
    return !(e && e[0] == '0');
  }();
  return v;
}
// LDS-DMA from inline asm (llmd_common.h glds16 / glds4) for the v3 kernel: hipcc then keeps
// counted lgkmcnt(N) waits for its fragment reads; the K loop's counted vmcnt covers them
__device__ __forceinline__ void g3_dma16(const void* src, char* lds_base) { glds16(src, lds_addr(lds_base)); }

template <int MODE, int POL = 0>
__global__ __launch_bounds__(G2_NT, 2) void moe_gemm2_kernel(
    const uint16_t* __restrict__ X, int64_t x_stride, int topk, const int* __restrict__ sorted_ids,
    const int* __restrict__ tile_expert, const uint16_t* __restrict__ W, int64_t w_expert_stride, int N, int K,
    uint16_t* __restrict__ Y, int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots,
    const uint16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(1024))) char buf0[G2_BUF];
  __shared__ __attribute__((aligned(1024))) char buf1[G2_BUF];
  const int mt = blockIdx.y, nt = blockIdx.x;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * G2_BM, n0 = nt * G2_BN;
  const uint16_t* We = W + (int64_t)e * w_expert_stride;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int lr = lane >> 3, lp = lane & 7;
  // DMA sources: A row groups {2w, 2w+1} (8 rows each), B row groups {8w .. 8w+7}
  const uint16_t* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (2 * w + i) + lr;
    const int sid = sorted_ids[m0 + row];
    const int tok = sid < 0 ? 0 : (a_rows_are_slots ? m0 + row : sid / topk);  // padding rows read row 0 (discarded)
    asrc[i] = X + (int64_t)tok * x_stride + g2_swz(row, lp) * 8;
  }
  const uint16_t* bsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (8 * w + i) + lr;
    const int n = min(n0 + row, N - 1);  // tail columns read a valid row (discarded)
    bsrc[i] = We + (int64_t)n * K + g2_swz(row, lp) * 8;
  }
  auto issue = [&](char* base, int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) g2_dma(asrc[i] + k0, base + (2 * w + i) * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) g2_dma<POL>(bsrc[i] + k0, base + G2_AB + (8 * w + i) * 1024);
  };
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, kq = lane >> 4;
  auto compute = [&](const char* base) {
    const char* A = base;
    const char* B = base + G2_AB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t af[4], bfr[4];
      const int c = 4 * s + kq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + r16;
        af[i] = *reinterpret_cast<const bf16x8_t*>(A + row * 128 + g2_swz(row, c) * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 64 * w + 16 * j + r16;
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(B + row * 128 + g2_swz(row, c) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nk = K / 64;
  issue(buf0, 0);
  for (int kt = 0; kt < nk; kt += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) issue(buf1, (kt + 1) * 64);
    compute(buf0);
    if (kt + 1 >= nk) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 2 < nk) issue(buf0, (kt + 2) * 64);
    compute(buf1);
  }
  // epilogue: C[row = 16i + 4kq + r][col = 64w + 16j + r16]
  // the expert bias of this lane's columns, loaded once (not once per accumulator element)
  float bvj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + 64 * w + 16 * j + r16;
    bvj[j] = (bias && col < N) ? bf2f(bias[(int64_t)e * N + col]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * i + kq * 4 + r;
      if (sorted_ids[row] < 0) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + 64 * w + 16 * j + r16;
        float v = acc[i][j][r];
        v += bvj[j];
        if (MODE == 0) {
          if (col < N) Y[(int64_t)row * y_stride + col] = f2bf(v);
        } else {
          const float other = __shfl_xor(v, 1, 64);
          if ((r16 & 1) == 0) {
            float g = v, u = other, o;
            if (act == 2) {
              g = fminf(g, limit);
              u = fminf(fmaxf(u, -limit), limit);
              o = (u + 1.f) * g / (1.f + __expf(-alpha * g));
            } else {
              o = g / (1.f + __expf(-g)) * u;
            }
            if (col < N) Y[(int64_t)row * y_stride + col / 2] = f2bf(o);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- FP8 grouped GEMM
// DeepGEMM role: e4m3fn operands with DeepSeek-style block
// scales - activations per (row, 128-K group) xs[row][kb], weights per
// (128-N x 128-K block) ws[e][nb][kb]. Same 64x128 tile and 4-wave layout as
// the bf16 kernel; a K-step is 128 fp8 = one scale block = the same 128-byte
// LDS row, so staging is byte-identical. Each K-step accumulates 4
// mfma_f32_16x16x32_fp8_fp8 into a block accumulator that is folded into the
// output accumulator with (xs[row][kb] * ws[e][nb][kb]) - exact block scaling,
// f32 accumulation. BN = 128 = the weight block height, so one weight scale per
// workgroup per K-step.
constexpr int BK8 = 128;
constexpr int LDA8 = BK8 + 16;  // bytes

template <int MODE>
__global__ __launch_bounds__(NT, 2) void moe_gemm_fp8_kernel(
    const uint8_t* __restrict__ X, int64_t x_stride, const float* __restrict__ xs, int64_t xs_stride, int topk,
    const int* __restrict__ sorted_ids, const int* __restrict__ tile_expert, const uint8_t* __restrict__ W,
    int64_t w_expert_stride, const float* __restrict__ ws, int N, int K, uint16_t* __restrict__ Y,
    int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots, const uint16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t As[2][BM][LDA8];
  __shared__ __attribute__((aligned(16))) uint8_t Bs[2][BN][LDA8];
  const int mt = blockIdx.y, nt = blockIdx.x;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nkb = (K + BK8 - 1) / BK8, nnb = (N + BN - 1) / BN;
  const uint8_t* We = W + (int64_t)e * w_expert_stride;
  const float* wse = ws + ((int64_t)e * nnb + nt) * nkb;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w >> 1, wn = w & 1;
  const int r16 = lane & 15, kq = lane >> 4;
  auto tok_of = [&](int row) {
    const int sid = sorted_ids[row];
    return sid < 0 ? -1 : (a_rows_are_slots ? row : sid / topk);
  };
  int arow[2], achk[2];
  const uint8_t* aptr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + NT * i;
    arow[i] = c >> 3;
    achk[i] = c & 7;
    const int tok = tok_of(m0 + arow[i]);
    aptr[i] = tok < 0 ? nullptr : X + (int64_t)tok * x_stride;
  }
  // activation-scale rows of this lane's output rows (i, r)
  const float* xsr[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tok = tok_of(m0 + wm * 32 + i * 16 + kq * 4 + r);
      xsr[i][r] = tok < 0 ? nullptr : xs + (int64_t)tok * xs_stride;
    }
  u32x4_t ra[2], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      u32x4_t v = {0, 0, 0, 0};
      if (aptr[i] && k0 + achk[i] * 16 < K) v = *reinterpret_cast<const u32x4_t*>(aptr[i] + k0 + achk[i] * 16);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      const int r = c >> 3, ch = c & 7;
      u32x4_t v = {0, 0, 0, 0};
      if (n0 + r < N && k0 + ch * 16 < K)
        v = *reinterpret_cast<const u32x4_t*>(We + (int64_t)(n0 + r) * K + k0 + ch * 16);
      rb[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4_t*>(&As[buf][arow[i]][achk[i] * 16]) = ra[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      *reinterpret_cast<u32x4_t*>(&Bs[buf][c >> 3][(c & 7) * 16]) = rb[i];
    }
  };
  f32x4_t acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nkb; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkb) load((kt + 1) * BK8);
    f32x4_t blk[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) blk[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < BK8 / 32; ++ks) {
      long af[2], bfr[4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const long*>(&As[buf][wm * 32 + i * 16 + r16][ks * 32 + kq * 8]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const long*>(&Bs[buf][wn * 64 + j * 16 + r16][ks * 32 + kq * 8]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) blk[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i], bfr[j], blk[i][j], 0, 0, 0);
    }
    const float wsv = wse[kt];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sc = xsr[i][r] ? xsr[i][r][kt] * wsv : 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j][r] += blk[i][j][r] * sc;
      }
    if (kt + 1 < nkb) {
      __syncthreads();
      store(buf ^ 1);
      __syncthreads();
    }
  }
  // the expert bias of this lane's columns, loaded once (not once per accumulator element)
  float bvj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + r16;
    bvj[j] = (bias && col < N) ? bf2f(bias[(int64_t)e * N + col]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm * 32 + i * 16 + kq * 4 + r;
      if (sorted_ids[row] < 0) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + r16;
        float v = acc[i][j][r];
        v += bvj[j];
        if (MODE == 0) {
          if (col < N) Y[(int64_t)row * y_stride + col] = f2bf(v);
        } else {
          const float other = __shfl_xor(v, 1, 64);
          if ((r16 & 1) == 0) {
            float g = v, u = other, o;
            if (act == 2) {
              g = fminf(g, limit);
              u = fminf(fmaxf(u, -limit), limit);
              o = (u + 1.f) * g / (1.f + __expf(-alpha * g));
            } else {
              o = g / (1.f + __expf(-g)) * u;
            }
            if (col < N) Y[(int64_t)row * y_stride + col / 2] = f2bf(o);
          }
        }
      }
    }
  }
}


// FP8 variant of the v2 grouped GEMM on the block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, unit E8M0 scales): one
// instruction per 16x16 tile per 128-K step at 2x the bf16 rate
// (MI355X_MICROARCH.md "FP8"). A K-step is 128 e4m3 = the same 128-B LDS row
// as the bf16 kernel, so the DMA staging is unchanged; lane l takes the 32
// bytes [32*(l>>4), +32) of its row (operand layout probed by
// scripts/probes/mfma_scale_layout.hip) with two ds_read_b128. The 16-B chunk
// swizzle is g3(row) = tab[(row>>1)&7], tab = {0,1,4,5,6,7,2,3}, which keeps
// both halves of those 32-B reads (and 16-B bf16-style reads) free of bank
// conflicts for all four ds_read_b128 lane groups. Each step's product is
// folded into the accumulator with xs[row][kb] * ws[e][nb][kb] (DeepSeek
// 1x128 activation / 128x128 weight block scales; each wave's 64 columns sit
// in one weight-scale block). The K loop issues no VGPR-destination load: the
// weight scale is a scalar load and the 64 activation scales of the next step
// ride the tile's LDS-DMA (a 4-byte global_load_lds per row) into their own
// per-buffer LDS array - an ordinary vector load there made hipcc wait
// vmcnt(0) inside every step, i.e. for the next tile's DMA too, serialising
// DMA and MFMAs (613 TF/s at T=4096, below the bf16 kernel).
__device__ __forceinline__ int g3_swz(int row, int c) { return c ^ ((0x32765410 >> (4 * ((row >> 1) & 7))) & 7); }

typedef int i32x8_t __attribute__((ext_vector_type(8)));

// HWS (hardware scales): the block scales are powers of two (quant_fp8_groups /
// quant_fp8_block_weight make them so), handed to the MFMA as E8M0 exponents -
// lane l's scale_a applies to A row l&15, scale_b to B column l&15, over the
// instruction's whole 128-deep K step when all four lane groups carry the same
// value (probed: scripts/probes/mfma_scale_map2.hip) - and the product is
// accumulated in place: no per-step block accumulator, no VALU re-scaling
// (~10 VALU per MFMA before), MFMAs back to back.
template <int MODE, bool HWS, int POL = 0>
__global__ __launch_bounds__(G2_NT, 2) void moe_gemm2_fp8_kernel(
    const uint8_t* __restrict__ X, int64_t x_stride, const float* __restrict__ xs, int64_t xs_stride, int topk,
    const int* __restrict__ sorted_ids, const int* __restrict__ tile_expert, const uint8_t* __restrict__ W,
    int64_t w_expert_stride, const float* __restrict__ ws, int N, int K, uint16_t* __restrict__ Y, int64_t y_stride,
    int act, float alpha, float limit, int a_rows_are_slots, const uint16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(1024))) char buf0[G2_BUF];
  __shared__ __attribute__((aligned(1024))) char buf1[G2_BUF];
  const int mt = blockIdx.y, nt = blockIdx.x;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * G2_BM, n0 = nt * G2_BN;
  const int nkb = K / 128, nnb = (N + 127) / 128;
  const uint8_t* We = W + (int64_t)e * w_expert_stride;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int lr = lane >> 3, lp = lane & 7;
  auto tok_of = [&](int row) {
    const int sid = sorted_ids[row];
    return sid < 0 ? -1 : (a_rows_are_slots ? row : sid / topk);
  };
  const uint8_t* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (2 * w + i) + lr;
    const int tok = tok_of(m0 + row);
    asrc[i] = X + (int64_t)(tok < 0 ? 0 : tok) * x_stride + g3_swz(row, lp) * 16;
  }
  int boff[8];  // 32-bit offsets into this expert's weights (fewer live VGPRs than 8 pointers)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (8 * w + i) + lr;
    const int n = min(n0 + row, N - 1);
    boff[i] = n * K + g3_swz(row, lp) * 16;
  }
  // Scales stay out of LDS so the kernel holds exactly two 40 KB tile buffers
  // (80 KB): two workgroups per CU. (Staging them in LDS - 1.5 KB more - left
  // one workgroup per CU and half the bytes in flight.) Lane r keeps the
  // activation scale xs[row r][kb] in a VGPR, loaded one K-step ahead right
  // after that step's DMA, so the loop-top vmcnt(0) covers it; rows are
  // fetched across lanes with ds_bpermute. The wave's weight-block scale is a
  // uniform (scalar) load, also one step ahead. Padding rows read row 0
  // (their outputs are never stored).
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const float* xs_row = xs + (int64_t)max(0, tok_of(m0 + lane)) * xs_stride;
  const float* wsr = ws + ((int64_t)e * nnb + (n0 + 64 * wu) / 128) * nkb;
  auto issue = [&](char* base, int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) g2_dma(asrc[i] + k0, base + (2 * w + i) * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) g2_dma<POL>(We + boff[i] + k0, base + G2_AB + (8 * w + i) * 1024);
  };
  const int r16 = lane & 15, kq = lane >> 4;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const char* base, float xv, float wsv) {
    const char* A = base;
    const char* B = base + G2_AB;
    i32x8_t bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 64 * w + 16 * j + r16;
      const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(B + row * 128 + g3_swz(row, 2 * kq) * 16);
      const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(B + row * 128 + g3_swz(row, 2 * kq + 1) * 16);
      bfr[j] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    if constexpr (HWS) {
      const int xe = e8m0_of(xv), we = e8m0_of(wsv);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + r16;
        const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(A + row * 128 + g3_swz(row, 2 * kq) * 16);
        const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(A + row * 128 + g3_swz(row, 2 * kq + 1) * 16);
        const i32x8_t af =
            i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        const int sa = __shfl(xe, row, 64);  // lane `row` holds the scale of tile row `row`
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], acc[i][j], 0, 0, 0, sa, 0, we);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // one 16-row block at a time keeps the block accumulators at 16 VGPRs
      const int row = 16 * i + r16;
      const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(A + row * 128 + g3_swz(row, 2 * kq) * 16);
      const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(A + row * 128 + g3_swz(row, 2 * kq + 1) * 16);
      const i32x8_t af =
          i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      f32x4_t blk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        blk[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0,
                                                                  127, 0, 127);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sc = __shfl(xv, 16 * i + 4 * kq + r, 64) * wsv;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j][r] += blk[j][r] * sc;
      }
    }
  };
  float xv0 = xs_row[0], wv0 = wsr[0];
  issue(buf0, 0);
  for (int kt = 0; kt < nkb; kt += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float xv1 = 0.f, wv1 = 0.f;
    if (kt + 1 < nkb) {
      issue(buf1, (kt + 1) * 128);
      xv1 = xs_row[kt + 1];
      wv1 = wsr[kt + 1];
    }
    compute(buf0, xv0, wv0);
    if (kt + 1 >= nkb) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 2 < nkb) {
      issue(buf0, (kt + 2) * 128);
      xv0 = xs_row[kt + 2];
      wv0 = wsr[kt + 2];
    }
    compute(buf1, xv1, wv1);
  }
  // the expert bias of this lane's columns, loaded once (not once per accumulator element)
  float bvj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + 64 * w + 16 * j + r16;
    bvj[j] = (bias && col < N) ? bf2f(bias[(int64_t)e * N + col]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * i + kq * 4 + r;
      if (sorted_ids[row] < 0) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + 64 * w + 16 * j + r16;
        float v = acc[i][j][r];
        v += bvj[j];
        if (MODE == 0) {
          if (col < N) Y[(int64_t)row * y_stride + col] = f2bf(v);
        } else {
          const float other = __shfl_xor(v, 1, 64);
          if ((r16 & 1) == 0) {
            float g = v, u = other, o;
            if (act == 2) {
              g = fminf(g, limit);
              u = fminf(fmaxf(u, -limit), limit);
              o = (u + 1.f) * g / (1.f + __expf(-alpha * g));
            } else {
              o = g / (1.f + __expf(-g)) * u;
            }
            if (col < N) Y[(int64_t)row * y_stride + col / 2] = f2bf(o);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- FP8 grouped GEMM v3 (prefill shapes)
// For steps where experts receive many rows (prefill: gpt-oss ~160 rows per
// expert at 5k tokens, DeepSeek EP8 ~1k). v2's 64-row tiles re-read an
// expert's whole weight panel once per 64 rows - at gpt-oss shapes three
// passes over 3.2 GB of weights per layer - and 64x256 tiles carry only 105
// FLOP per staged byte. v3 takes 256-row expert tiles (moe_align with
// bm = 256: one tile holds every row of a gpt-oss expert) x 256 columns on
// ONE 512-thread workgroup per CU:
//   * 8 waves as 2 (M) x 4 (N), each 128 x 64 = 4 x 2 tiles of
//     v_mfma_scale_f32_32x32x64_f8f6f4 (128 accumulator VGPRs; layout probed by
//     scripts/probes/mfma32_scale_layout.hip); E8M0 hardware block scales
//     (power-of-two scales, see HWS above): the K loop is MFMAs, fragment
//     reads and DMA issue only;
//   * K-steps of 64 fp8 through a 4-deep LDS ring (34 KB per stage: A 256 x
//     64 B gathered through sorted_ids by the DMA's per-lane source address,
//     B 256 x 64 B, and the step's activation scales, which ride the DMA too:
//     an ordinary vector load in the loop would make hipcc drain vmcnt(0)),
//     three stages in flight across raw s_barriers with COUNTED vmcnt waits;
//     64-B rows, 16-B chunks XOR-swizzled by (row >> 2) & 3 on the DMA source
//     so every ds_read_b128 lane group covers 16 distinct bank slots;
//   * rows past the expert's last row (moe_align pads experts to 256) are
//     loaded (from token 0, L2 hits: the DMA count per stage stays fixed for
//     the counted waits) but not multiplied or stored: the valid rows are a
//     prefix, each wave skips its 32-row blocks past it (wave-uniform).
// BF (bf16 operands, round 4): the same 64-B image rows hold 32 bf16 = one
// K-step of two v_mfma_f32_32x32x16_bf16 per 32x32 tile (lane half h reads
// chunks h and 2 + h, conflict-free under the same swizzle), no scales, four
// DMA pieces per wave per stage.
constexpr int G3_BM = 256, G3_BN = 256, G3_NT = 512, G3_NS = 4;
constexpr int G3_A = G3_BM * 64, G3_B = G3_BN * 64, G3_SC = 8 * 256;
constexpr int G3_STAGE = G3_A + G3_B + G3_SC;  // 34 KB
constexpr int G3_OPS = 5;                       // VMEM ops per wave per stage: 2 A + 2 B + 1 scale

typedef float f32x16v_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int g3r_swz(int row, int c) { return c ^ ((row >> 2) & 3); }

__device__ __forceinline__ void g3_dma4(const void* src, char* lds_base) { glds4(src, lds_addr(lds_base)); }

// FQ (MODE 1 only): the gated activation's output is quantised in the epilogue
// straight to the second GEMM's fp8 operand - one workgroup's 256 gate/up
// columns are exactly one 128-column activation-scale group, so the row amax
// needs only the four N-waves' partials (exchanged through the then idle LDS
// ring) - instead of a bf16 h round trip through HBM and a quant_fp8_groups
// pass over every padded row. Same numerics as that pass: the bf16-rounded
// value, power-of-two scale pow2_ceil(max(amax / 448, 1e-12)), saturating e4m3.
// Ablation switch for profiling (LLMD_MOE_ABLATE: 1 = no MFMA / fragment reads,
// 2 = no DMA after the prologue); 0 in production.
__device__ int g3_ablate = 0;
__device__ int g3_xcd = 0;

// V (fp8 A/B switch, round 4): bit 0 = A fragments read one row block ahead,
// bit 1 = LDS-DMA from asm (glds16/glds4) instead of the builtin
template <int MODE, bool FQ, bool BF = false, int V = 3>
__global__ __launch_bounds__(G3_NT, 1) void moe_gemm3_fp8_kernel(
    const uint8_t* __restrict__ X, int64_t x_stride, const float* __restrict__ xs, int64_t xs_stride, int topk,
    const int* __restrict__ sorted_ids, const int* __restrict__ tile_expert, const uint8_t* __restrict__ W,
    int64_t w_expert_stride, const float* __restrict__ ws, int N, int K, uint16_t* __restrict__ Y, int64_t y_stride,
    int act, float alpha, float limit, int a_rows_are_slots, const uint16_t* __restrict__ bias,
    uint8_t* __restrict__ hq, int64_t hq_stride, float* __restrict__ hs, int64_t hs_stride) {
  // ONE __shared__ array (a second LDS object can make hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(1024))) char lds[G3_NS * G3_STAGE];
  // g3_xcd (LLMD_MOE_V3_XCD=1): deal tiles to XCDs in contiguous runs (xcd_remap) so the N tiles
  // of one 256-row A panel share that XCD's L2 instead of every XCD fetching the panel
  int mt = blockIdx.y, nt = blockIdx.x;
  if (g3_xcd) {
    const int l = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    nt = l % gridDim.x;
    mt = l / gridDim.x;
  }
  const int e = tile_expert[mt];
  if (e < 0) return;
  static_assert(!(FQ && BF), "fused quantisation is an fp8-path epilogue");
  const int m0 = mt * G3_BM, n0 = nt * G3_BN;
  constexpr int EB = BF ? 2 : 1;  // bytes per element; a K-step is 64 B of every row
  const int nk = K * EB / 64, nkb = K / 128, nnb = (N + 127) / 128;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w >> 2, wn = w & 3;
  const int l32 = lane & 31, h = lane >> 5;
  // valid rows of this tile (a prefix: moe_align pads each expert at its end), counted per wave
  // with ballots: no LDS object besides the staging ring (a second one, like __syncthreads_count's,
  // makes hipcc wait vmcnt(0) for the in-flight DMAs before every ds_read)
  int nvalid = 0;
#pragma unroll
  for (int q = 0; q < G3_BM / 64; ++q) nvalid += __popcll(__ballot(sorted_ids[m0 + 64 * q + lane] >= 0));
  auto tok_of = [&](int row) {
    const int sid = sorted_ids[row];
    return sid < 0 ? -1 : (a_rows_are_slots ? row : sid / topk);
  };
  // DMA sources: a 1 KB piece = 16 rows x 64 B; wave w moves A pieces {2w, 2w+1}, B pieces {2w, 2w+1}
  // and the activation scales of rows 32w + (lane & 31)
  const int lr = lane >> 2, lp = lane & 3;
  int aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (2 * w + i) + lr;
    const int tok = tok_of(m0 + row);
    aoff[i] = (tok < 0 ? 0 : tok) * (int)x_stride * EB + g3r_swz(row, lp) * 16;
    boff[i] = min(n0 + row, N - 1) * K * EB + g3r_swz(row, lp) * 16;  // tail columns: a valid row, never stored
  }
  const int stok = tok_of(m0 + 32 * w + l32);
  const float* xsr = xs + (int64_t)(stok < 0 ? 0 : stok) * xs_stride;
  const uint8_t* We = W + (int64_t)e * w_expert_stride * EB;
  auto issue = [&](int kt) {
    char* st = lds + (kt & (G3_NS - 1)) * G3_STAGE;
    const int k0 = kt * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (V & 2) g3_dma16(X + aoff[i] + k0, st + (2 * w + i) * 1024);
      else g2_dma(X + aoff[i] + k0, st + (2 * w + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr ((V & 6) == 6) glds16_nt(We + boff[i] + k0, lds_addr(st + G3_A + (2 * w + i) * 1024));
      else if constexpr (V & 2) g3_dma16(We + boff[i] + k0, st + G3_A + (2 * w + i) * 1024);
      else g2_dma(We + boff[i] + k0, st + G3_A + (2 * w + i) * 1024);
    }
    if constexpr (!BF) {
      if constexpr (V & 2) g3_dma4(xsr + (kt >> 1), st + G3_A + G3_B + w * 256);
      else __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(xsr + (kt >> 1)),
                                            (void __attribute__((address_space(3)))*)(st + G3_A + G3_B + w * 256),
                                            4, 0, 0);
    }
  };
  const float* wsr = BF ? nullptr : ws + ((int64_t)e * nnb + (n0 + 64 * __builtin_amdgcn_readfirstlane(wn)) / 128) * nkb;
  // wave wm owns the 32-row blocks {wm, wm + 2, wm + 4, wm + 6} (interleaved: an expert with
  // ~160 rows gives the two halves 3 and 2 blocks, not 4 and 1); live = blocks before nvalid
  const int nblk = (nvalid + 31) / 32;
  const int rb_live = min(4, max(0, (nblk - wm + 1) / 2));
  // fragment reads: lane (l32, h) takes row l32 of a 32-row block, bytes [32h, 32h+32) = chunks 2h, 2h+1;
  // the swizzle key (row >> 2) & 3 is the same for every 32-row block
  // (bf16: k-substep 0 reads chunk h, k-substep 1 chunk 2 + h)
  const int sw_lo = g3r_swz(l32, BF ? h : 2 * h) * 16, sw_hi = g3r_swz(l32, BF ? 2 + h : 2 * h + 1) * 16;
  const int a_off = (32 * wm + l32) * 64, b_off = G3_A + (64 * wn + l32) * 64;  // block i: + i * 4096
  const int s_off = G3_A + G3_B + wm * 256 + l32 * 4;  // scale of row 32*(wm + 2i) + l32: + i * 512
  f32x16v_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16v_t{};
  const int ablate = __builtin_amdgcn_readfirstlane(g3_ablate);
  auto compute = [&](int kt, bool refill) {
    if (ablate) {
      if (refill && !(ablate & 2)) issue(kt + G3_NS - 1);
      if (ablate & 1) return;
      refill = false;
    }
    const char* st = lds + (kt & (G3_NS - 1)) * G3_STAGE;
    if constexpr (BF) {
      bf16x8_t bfr[2][2];  // [col block][k-substep]
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bfr[j][0] = *reinterpret_cast<const bf16x8_t*>(st + b_off + j * 2048 + sw_lo);
        bfr[j][1] = *reinterpret_cast<const bf16x8_t*>(st + b_off + j * 2048 + sw_hi);
      }
      bf16x8_t a_cur[2], a_nxt[2];
      if ((V & 1) && rb_live > 0) {
        a_cur[0] = *reinterpret_cast<const bf16x8_t*>(st + a_off + sw_lo);
        a_cur[1] = *reinterpret_cast<const bf16x8_t*>(st + a_off + sw_hi);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i >= rb_live) break;  // wave-uniform: 32-row blocks past the expert's rows
        if constexpr (V & 1) {
          if (i + 1 < rb_live) {
            a_nxt[0] = *reinterpret_cast<const bf16x8_t*>(st + a_off + (i + 1) * 4096 + sw_lo);
            a_nxt[1] = *reinterpret_cast<const bf16x8_t*>(st + a_off + (i + 1) * 4096 + sw_hi);
          }
        } else {
          a_cur[0] = *reinterpret_cast<const bf16x8_t*>(st + a_off + i * 4096 + sw_lo);
          a_cur[1] = *reinterpret_cast<const bf16x8_t*>(st + a_off + i * 4096 + sw_hi);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_cur[ks], bfr[j][ks], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (i == 0 && refill) issue(kt + G3_NS - 1);
        if constexpr (V & 1) {
          a_cur[0] = a_nxt[0];
          a_cur[1] = a_nxt[1];
        }
      }
    } else {
      const int we = e8m0_of(wsr[kt >> 1]);
      i32x8_t bfr[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(st + b_off + j * 2048 + sw_lo);
        const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(st + b_off + j * 2048 + sw_hi);
        bfr[j] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
      auto aread = [&](int i, i32x8_t& af, float& sc) {
        const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(st + a_off + i * 4096 + sw_lo);
        const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(st + a_off + i * 4096 + sw_hi);
        af = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        sc = *reinterpret_cast<const float*>(st + s_off + i * 512);
      };
      // block i's A fragment is read one block ahead of its MFMAs (counted lgkmcnt waits:
      // the DMA is asm, g3_dma16), so a read's latency hides behind the previous block's MFMAs
      i32x8_t af_cur, af_nxt;
      float sc_cur = 0.f, sc_nxt = 0.f;
      if ((V & 1) && rb_live > 0) aread(0, af_cur, sc_cur);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i >= rb_live) break;  // wave-uniform: 32-row blocks past the expert's rows
        if constexpr (V & 1) {
          if (i + 1 < rb_live) aread(i + 1, af_nxt, sc_nxt);
        } else {
          aread(i, af_cur, sc_cur);  // read right before its MFMAs (round-3 schedule)
        }
        const int sa = e8m0_of(sc_cur);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af_cur, bfr[j], acc[i][j], 0, 0, 0, sa, 0, we);
        __builtin_amdgcn_sched_barrier(0);
        // the next stage's DMA issues behind the first block's MFMAs (they start the matrix pipe at once)
        if (i == 0 && refill) issue(kt + G3_NS - 1);
        if constexpr (V & 1) {
          af_cur = af_nxt;
          sc_cur = sc_nxt;
        }
      }
    }
    if (rb_live == 0 && refill) issue(kt + G3_NS - 1);
  };
#pragma unroll
  for (int s = 0; s < G3_NS - 1; ++s)
    if (s < nk) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (this wave's DMAs; the barrier extends it to every wave's), and every
    // wave is done reading the stage that issue(kt + 3) overwrites (it was read in step kt - 1)
    // G3_OPS (fp8) or 4 (bf16, no scale piece) DMA ops per wave per stage
    if (kt + 2 < nk) {
      if constexpr (BF) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else if (kt + 1 < nk) {
      if constexpr (BF) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(kt, kt + G3_NS - 1 < nk);
  }
  // epilogue: acc[i][j][r] = C[row 32*(wm + 2i) + (r&3) + 8(r>>2) + 4h][col 64*wn + 32j + l32]
  if constexpr (FQ && MODE == 1) {
    // pass 1: bias + gated activation in place (even lanes hold o, odd lanes 0), per-row amax of
    // this wave's 32 h columns, partials of the 4 N-waves through LDS
    __syncthreads();  // every wave is out of the K loop: the ring is free
    float* amax_lds = reinterpret_cast<float*>(lds);  // [256 rows][4 N-waves]
    // the expert bias of this lane's columns, loaded once (not once per accumulator element)
    float bvj[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + 64 * wn + 32 * j + l32;
      bvj[j] = (bias && col < N) ? bf2f(bias[(int64_t)e * N + col]) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + 64 * wn + 32 * j + l32;
          float v = acc[i][j][r];
          v += bvj[j];
          const float other = __shfl_xor(v, 1, 64);
          float o = 0.f;
          if ((l32 & 1) == 0 && col < N) {
            float g = v, u = other;
            if (act == 2) {
              g = fminf(g, limit);
              u = fminf(fmaxf(u, -limit), limit);
              o = (u + 1.f) * g / (1.f + __expf(-alpha * g));
            } else {
              o = g / (1.f + __expf(-g)) * u;
            }
            o = bf2f(f2bf(o));  // the value the unfused path would have stored
          }
          acc[i][j][r] = o;
          a = fmaxf(a, fabsf(o));
        }
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) a = fmaxf(a, __shfl_xor(a, off, 64));
        if (l32 == 0) amax_lds[(32 * (wm + 2 * i) + (r & 3) + 8 * (r >> 2) + 4 * h) * 4 + wn] = a;
      }
    }
    __syncthreads();
    // pass 2: scale per row, e4m3 bytes of this workgroup's 128-column group (zeros past F)
    const int hc0 = n0 / 2 + 32 * wn + l32 / 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= rb_live) break;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = 32 * (wm + 2 * i) + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int row = m0 + rl;
        if (sorted_ids[row] < 0) continue;
        const float* am = amax_lds + rl * 4;
        const float s = pow2_ceil(fmaxf(fmaxf(fmaxf(am[0], am[1]), fmaxf(am[2], am[3])) / FP8_MAX, 1e-12f));
        const float inv = 1.f / s;
        if ((l32 & 1) == 0) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float c = fminf(fmaxf(acc[i][j][r] * inv, -FP8_MAX), FP8_MAX);
            hq[(int64_t)row * hq_stride + hc0 + 16 * j] =
                (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(c, 0.f, 0, false) & 0xff);
          }
        }
        if (wn == 0 && l32 == 0) hs[(int64_t)row * hs_stride + nt] = s;
      }
    }
    return;
  }
  // the expert bias of this lane's columns, loaded once (not once per accumulator element)
  float bvj[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + 64 * wn + 32 * j + l32;
    bvj[j] = (bias && col < N) ? bf2f(bias[(int64_t)e * N + col]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= rb_live) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + 32 * (wm + 2 * i) + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool live = sorted_ids[row] >= 0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + 64 * wn + 32 * j + l32;
        float v = acc[i][j][r];
        v += bvj[j];
        if (MODE == 0) {
          if (live && col < N) Y[(int64_t)row * y_stride + col] = f2bf(v);
        } else {
          const float other = __shfl_xor(v, 1, 64);
          if (live && (l32 & 1) == 0) {
            float g = v, u = other, o;
            if (act == 2) {
              g = fminf(g, limit);
              u = fminf(fmaxf(u, -limit), limit);
              o = (u + 1.f) * g / (1.f + __expf(-alpha * g));
            } else {
              o = g / (1.f + __expf(-g)) * u;
            }
            if (col < N) Y[(int64_t)row * y_stride + col / 2] = f2bf(o);
          }
        }
      }
    }
  }
}

// out[t, :] = sum_j w[t, j] * Y[pos(t, j), :]  with pos from the inverse permutation
__global__ __launch_bounds__(256) void moe_combine_kernel(const uint16_t* __restrict__ Y, int64_t y_stride,
                                                          const int* __restrict__ inv, const float* __restrict__ w,
                                                          int topk, int d, uint16_t* __restrict__ out,
                                                          int64_t out_stride) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < d / 8; c += 256) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < topk; ++j) {
      const int p = inv[(int64_t)t * topk + j];
      if (p < 0) continue;
      const float ww = w[(int64_t)t * topk + j];
      float f[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(Y + (int64_t)p * y_stride + c * 8), f);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += ww * f[q];
    }
    *reinterpret_cast<u32x4_t*>(out + (int64_t)t * out_stride + c * 8) = pack8(acc);
  }
}

__global__ void moe_invert_kernel(const int* __restrict__ sorted_ids, int P, int* __restrict__ inv) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P) {
    const int s = sorted_ids[p];
    if (s >= 0) inv[s] = p;
  }
}

}  // namespace

extern "C" {

void llmd_moe_topk(const float* logits, int T, int E, int K, int scoring, const float* bias, int n_group,
                   int topk_group, int renorm, float routed_scale, int* ids, float* wts, hipStream_t st) {
  if (T == 0) return;
  hipLaunchKernelGGL(moe_topk_kernel, dim3((T + 3) / 4), dim3(256), 0, st, logits, T, E, K, scoring, bias,
                     n_group, topk_group, renorm, routed_scale, ids, wts);
}

// max_p = n + E*(BM-1) rounded to BM
void llmd_moe_align(const int* ids, int n, int E, int bm, int* sorted_ids, int* tile_expert,
                    int* expert_offsets, int max_p, int* total_p, int* inv, hipStream_t st) {
  const size_t lds = (size_t)(3 * E + 1) * sizeof(int);
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(1024), lds, st, ids, n, E, bm, sorted_ids, tile_expert,
                     expert_offsets, max_p, total_p, inv);
  hipLaunchKernelGGL(moe_invert_kernel, dim3((max_p + 255) / 256), dim3(256), 0, st, sorted_ids, max_p, inv);
}

int llmd_moe_gemm_tile_m() { return BM; }

void llmd_moe_gemm(const void* X, int64_t x_stride, int topk, const int* sorted_ids, const int* tile_expert,
                   int num_tiles, const void* W, int64_t w_expert_stride, int N, int K, void* Y, int64_t y_stride,
                   int mode, int act, float alpha, float limit, int a_rows_are_slots, const void* bias,
                   hipStream_t st) {
  if (num_tiles == 0) return;
  static const bool v2 = [] {
    const char* e = getenv("LLMD_MOE_GEMM_V1");
    return !(e && e[0] == '1');
  }();
  if (v2 && K % 64 == 0 && (x_stride % 8) == 0 && (w_expert_stride % 8) == 0) {
    dim3 grid2((N + G2_BN - 1) / G2_BN, num_tiles);
    const bool nt = moe_nt();
    if (mode == 0)
      hipLaunchKernelGGL((nt ? moe_gemm2_kernel<0, 2> : moe_gemm2_kernel<0, 0>), grid2, dim3(G2_NT), 0, st, (const uint16_t*)X, x_stride, topk,
                         sorted_ids, tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y, y_stride,
                         act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias);
    else
      hipLaunchKernelGGL((nt ? moe_gemm2_kernel<1, 2> : moe_gemm2_kernel<1, 0>), grid2, dim3(G2_NT), 0, st, (const uint16_t*)X, x_stride, topk,
                         sorted_ids, tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y, y_stride,
                         act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias);
    return;
  }
  dim3 grid((N + BN - 1) / BN, num_tiles);
  if (mode == 0)
    hipLaunchKernelGGL(moe_gemm_kernel<0>, grid, dim3(NT), 0, st, (const uint16_t*)X, x_stride, topk, sorted_ids,
                       tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y, y_stride, act, alpha,
                       limit, a_rows_are_slots, (const uint16_t*)bias);
  else
    hipLaunchKernelGGL(moe_gemm_kernel<1>, grid, dim3(NT), 0, st, (const uint16_t*)X, x_stride, topk, sorted_ids,
                       tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y, y_stride, act, alpha,
                       limit, a_rows_are_slots, (const uint16_t*)bias);
}

int llmd_moe_gemm3_tile_m() { return G3_BM; }

// LLMD_MOE_V3_NT=1: the v3 expert-weight DMA with the nt policy (schedule variant 2 only; A/B)
static bool g3_nt() {
  static const bool v = [] {
    const char* e = getenv("LLMD_MOE_V3_NT");
    return e && e[0] == '1';
  }();
  return v;
}

// device-side switches of the v3 kernels, read from the environment once per process
static void g3_env() {
  static const bool done = [] {
    const char* e = getenv("LLMD_MOE_ABLATE");
    const int v = e ? atoi(e) : 0;
    if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(g3_ablate), &v, sizeof v);
    const char* x = getenv("LLMD_MOE_V3_XCD");
    const int xv = x ? atoi(x) : 0;
    if (xv) (void)hipMemcpyToSymbol(HIP_SYMBOL(g3_xcd), &xv, sizeof xv);
    return true;
  }();
  (void)done;
}

// 256-row expert tiles (sorted by moe_align with bm = 256): the v3 kernel.
// Needs power-of-two scales, K % 128 == 0 and 16-B aligned rows.
// hq != nullptr (mode 1): fused e4m3 quantisation of the activation output into hq
// [rows, >= N/2 rounded to 128] with power-of-two scales hs [rows, N/256 groups].
int llmd_moe_gemm3_fp8(const void* X, int64_t x_stride, const float* xs, int64_t xs_stride, int topk,
                       const int* sorted_ids, const int* tile_expert, int num_tiles, const void* W,
                       int64_t w_expert_stride, const float* ws, int N, int K, void* Y, int64_t y_stride, int mode,
                       int act, float alpha, float limit, int a_rows_are_slots, const void* bias, void* hq,
                       int64_t hq_stride, float* hs, int64_t hs_stride, hipStream_t st) {
  if (K % 128 || x_stride % 16 || w_expert_stride % 16) return -1;
  if (hq && mode != 1) return -2;
  g3_env();
  if (num_tiles == 0) return 0;
  dim3 grid((N + G3_BN - 1) / G3_BN, num_tiles);
  static const int g3v = [] {
    // A/B of the round-4 fp8 v3 schedule (V above; profiles/moe_gemm_v3_r4_ab.txt): the A prefetch
    // lost 6 % (DeepSeek EP8 T=4096 2.20 -> 2.35 ms), the asm DMA alone is at parity or better -> 2
    const char* e = getenv("LLMD_MOE_V3_VARIANT");
    return e ? (atoi(e) & 3) : 2;
  }();
#define LLMD_G3F8(M, Q)                                                                                           \
  do {                                                                                                            \
    if (g3v == 2 && g3_nt()) LLMD_G3F8V(M, Q, 6); else                                                          \
    if (g3v == 0) LLMD_G3F8V(M, Q, 0); else if (g3v == 1) LLMD_G3F8V(M, Q, 1);                                  \
    else if (g3v == 2) LLMD_G3F8V(M, Q, 2); else LLMD_G3F8V(M, Q, 3);                                           \
  } while (0)
#define LLMD_G3F8V(M, Q, VV)                                                                                      \
  hipLaunchKernelGGL((moe_gemm3_fp8_kernel<M, Q, false, VV>), grid, dim3(G3_NT), 0, st, (const uint8_t*)X,       \
                     x_stride, xs,                                                                                 \
                     xs_stride, topk, sorted_ids, tile_expert, (const uint8_t*)W, w_expert_stride, ws, N, K,       \
                     (uint16_t*)Y, y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias,           \
                     (uint8_t*)hq, hq_stride, hs, hs_stride)
  if (mode == 0) LLMD_G3F8(0, false);
  else if (hq) LLMD_G3F8(1, true);
  else LLMD_G3F8(1, false);
#undef LLMD_G3F8
#undef LLMD_G3F8V
  return (int)hipGetLastError();
}

// bf16 operands on the v3 tiles (256-row expert tiles from moe_align with bm = 256)
int llmd_moe_gemm3_bf16(const void* X, int64_t x_stride, int topk, const int* sorted_ids, const int* tile_expert,
                        int num_tiles, const void* W, int64_t w_expert_stride, int N, int K, void* Y, int64_t y_stride,
                        int mode, int act, float alpha, float limit, int a_rows_are_slots, const void* bias,
                        hipStream_t st) {
  if (K % 32 || x_stride % 8 || w_expert_stride % 8) return -1;
  g3_env();
  if (num_tiles == 0) return 0;
  dim3 grid((N + G3_BN - 1) / G3_BN, num_tiles);
  static const int bfv = [] {  // schedule variant for bf16 (bits as V; LLMD_MOE_V3_BF16_VARIANT)
    // A/B (profiles/moe_gemm_v3_r4_ab.txt): without the A prefetch DeepSeek EP8 T=4096 794 -> 821 TF/s
    const char* e = getenv("LLMD_MOE_V3_BF16_VARIANT");
    return e ? (atoi(e) & 3) : 2;
  }();
#define LLMD_G3BF(M)                                                                                              \
  do {                                                                                                            \
    if (bfv == 2 && g3_nt()) LLMD_G3BFV(M, 6); else                                                             \
    if (bfv == 0) LLMD_G3BFV(M, 0); else if (bfv == 1) LLMD_G3BFV(M, 1);                                        \
    else if (bfv == 2) LLMD_G3BFV(M, 2); else LLMD_G3BFV(M, 3);                                                 \
  } while (0)
#define LLMD_G3BFV(M, VV)                                                                                         \
  hipLaunchKernelGGL((moe_gemm3_fp8_kernel<M, false, true, VV>), grid, dim3(G3_NT), 0, st, (const uint8_t*)X, x_stride, \
                     nullptr, 0, topk, sorted_ids, tile_expert, (const uint8_t*)W, w_expert_stride, nullptr, N, K,  \
                     (uint16_t*)Y, y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias, nullptr, 0, \
                     nullptr, 0)
  if (mode == 0) LLMD_G3BF(0);
  else LLMD_G3BF(1);
#undef LLMD_G3BF
#undef LLMD_G3BFV
  return (int)hipGetLastError();
}

void llmd_moe_gemm_fp8(const void* X, int64_t x_stride, const float* xs, int64_t xs_stride, int topk,
                       const int* sorted_ids, const int* tile_expert, int num_tiles, const void* W,
                       int64_t w_expert_stride, const float* ws, int N, int K, void* Y, int64_t y_stride, int mode,
                       int act, float alpha, float limit, int a_rows_are_slots, const void* bias, hipStream_t st) {
  if (num_tiles == 0) return;
  static const bool v2 = [] {
    const char* e = getenv("LLMD_MOE_GEMM_V1");
    return !(e && e[0] == '1');
  }();
  // power-of-two scales (every quantiser of this code base) run on the MFMA's
  // own E8M0 scales; LLMD_MOE_FP8_SOFT_SCALE=1 keeps the VALU block re-scaling
  static const bool hws = [] {
    const char* e = getenv("LLMD_MOE_FP8_SOFT_SCALE");
    return !(e && e[0] == '1');
  }();
  if (v2 && K % 128 == 0 && K / 128 <= G2_MAX_KB && x_stride % 16 == 0 && w_expert_stride % 16 == 0) {
    dim3 grid2((N + G2_BN - 1) / G2_BN, num_tiles);
    const bool nt = moe_nt();
#define LLMD_G2F8(M, H)                                                                                           \
  hipLaunchKernelGGL((nt ? moe_gemm2_fp8_kernel<M, H, 2> : moe_gemm2_fp8_kernel<M, H, 0>), grid2, dim3(G2_NT), 0, st, (const uint8_t*)X, x_stride, xs,     \
                     xs_stride, topk, sorted_ids, tile_expert, (const uint8_t*)W, w_expert_stride, ws, N, K,       \
                     (uint16_t*)Y, y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias)
    if (mode == 0) {
      if (hws) LLMD_G2F8(0, true);
      else LLMD_G2F8(0, false);
    } else {
      if (hws) LLMD_G2F8(1, true);
      else LLMD_G2F8(1, false);
    }
#undef LLMD_G2F8
    return;
  }
  dim3 grid((N + BN - 1) / BN, num_tiles);
  if (mode == 0)
    hipLaunchKernelGGL(moe_gemm_fp8_kernel<0>, grid, dim3(NT), 0, st, (const uint8_t*)X, x_stride, xs, xs_stride,
                       topk, sorted_ids, tile_expert, (const uint8_t*)W, w_expert_stride, ws, N, K, (uint16_t*)Y,
                       y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias);
  else
    hipLaunchKernelGGL(moe_gemm_fp8_kernel<1>, grid, dim3(NT), 0, st, (const uint8_t*)X, x_stride, xs, xs_stride,
                       topk, sorted_ids, tile_expert, (const uint8_t*)W, w_expert_stride, ws, N, K, (uint16_t*)Y,
                       y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias);
}

void llmd_moe_combine(const void* Y, int64_t y_stride, const int* inv, const float* w, int T, int topk, int d,
                      void* out, int64_t out_stride, hipStream_t st) {
  if (T == 0) return;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, st, (const uint16_t*)Y, y_stride, inv, w, topk,
                     d, (uint16_t*)out, out_stride);
}
}
