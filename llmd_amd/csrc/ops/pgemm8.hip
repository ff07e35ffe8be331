// Prefill ("large-M") fp8 W8A8 GEMM: C[M, N] = (xs . A[M, K]) (ws . W[N, K])^T,
// A and W e4m3fn, xs per-token and ws per-output-channel fp32 scales, bf16 C
// (SURVEY K08 + K16; the role of hipBLASLt's row-wise-scaled F8 GEMM behind
// torch._scaled_mm, which the reference's AMD P/D recipe runs for
// amd/Llama-3.3-70B-Instruct-FP8-KV, guides/pd-disaggregation/modelserver/amd/
// vllm/base/patch-decode.yaml:13).
//
// CDNA4 design - the bf16 PGR2 kernel (pgemm.hip variant 3) re-cut for the
// block-scaled MFMA, whose e4m3 form runs at twice the bf16 rate per clock:
//   * one 256 x 256 output tile per 4-wave workgroup, a wave owns 128 x 128 as
//     8 x 8 v_mfma_scale_f32_16x16x128_f8f6f4 tiles (256 AGPR accumulators);
//     the E8M0 scale operands are 1.0 and the fp32 scales are applied in the
//     epilogue, so the operands are exactly hipBLASLt's;
//   * a K-step is 128 fp8 = 128 B per row, i.e. byte-for-byte the bf16 PGR2
//     LDS image: 2 x 64 KB buffers, 1 KB LDS-DMA pieces (buffer_load ... lds,
//     K offset in soffset), 16-B chunks XOR-swizzled by row on the source side;
//   * one 16x16x128 MFMA consumes a whole K-step per fragment pair (32 B per
//     lane = 2 ds_read_b128), so there is no second k-half to pipeline
//     against. The schedule instead pipelines ACROSS steps: the W fragments
//     of step kt+1 go to a second register set (named statically by a 2-step
//     unroll), an A fragment is refilled in place once its row of 8 MFMAs is
//     done; per step (64 MFMA slots of 32 cycles):
//       t 1-2   A fragment 7 of THIS step (its register was busy until the end
//               of the previous step)
//       t 5     lgkmcnt(0) + barrier: every wave is done with this buffer
//       t 6-21  the 16 DMA pieces of step kt+2 into it
//       t 27    vmcnt(16) + barrier: step kt+1 landed
//       t 28-43 W fragments of step kt+1 (second set), t 44-55 A fragments
//               0-5 of step kt+1, t 57-58 A fragment 6
//     so a DMA piece has ~1.3 steps to land and LDS traffic is ~96 B/clk/CU;
//   * XCD-aware grouped tile order as pgemm.hip;
//   * epilogue through the free LDS (C^T: W fragments are the MFMA's A
//     operand, a lane holds 4 consecutive N columns of one token row), scaled
//     by xs[m] * ws[n] in fp32; EPI_SILU_STD fuses silu(gate) * up on the
//     model's plain [gate; up] weight (tile tn: gate rows [128 tn, +128),
//     up rows [F + 128 tn, +128)).
//
// Requirements (host-checked): N % 256 == 0, K % 128 == 0, 16-B aligned rows,
// byte offsets within 31 bits; any M (rows past M read zeros, not stored).
#include <algorithm>
#include <type_traits>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int P8_BM = 256, P8_BN = 256, P8_BK = 128, P8_NT = 256;
constexpr int P8_OPB = P8_BM * P8_BK;  // 32 KB per operand per K-step
constexpr int P8_BUF = 2 * P8_OPB;     // 64 KB
constexpr int P8_GROUP_M = 8;
constexpr uint32_t P8_OOB = 0x80000000u;  // past the 0x7fffffff buffer range: reads zeros

enum { P8_EPI_NONE = 0, P8_EPI_F32 = 2, P8_EPI_SILU_STD = 3 };

typedef int i32x8_t __attribute__((ext_vector_type(8)));

// D(16x16, f32) += A(16x128 e4m3) . B(128x16 e4m3), E8M0 scales 127 = 1.0
__device__ __forceinline__ void mfma8(f32x4_t& acc, const i32x8_t& a, const i32x8_t& b, int one) {
  asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
               : "+a"(acc)
               : "v"(a), "v"(b), "v"(one));
}

__device__ __forceinline__ void p8_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void p8_tile_mn(int L, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = P8_GROUP_M * tiles_n;
  const int g = L / per_group, first_m = g * P8_GROUP_M;
  const int gm = min(tiles_m - first_m, P8_GROUP_M);
  tm = first_m + (L % per_group) % gm;
  tn = (L % per_group) / gm;
}

template <int EPI>
__global__ __launch_bounds__(P8_NT, 1) void pgemm8_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ xs,
                                                          const uint8_t* __restrict__ W, int64_t ldw,
                                                          const float* __restrict__ wsc,
                                                          uint16_t* __restrict__ C, int64_t ldc, int M, int N,
                                                          int K, int tile0, int nsplit, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * P8_BUF];  // the ONLY LDS object
  const int tiles_m = (M + P8_BM - 1) / P8_BM, tiles_n = N / P8_BN;
  // nsplit > 1 (EPI_F32): the grid covers `tail` tiles from tile0 x nsplit K-ranges, each block
  // writing its scaled fp32 partial tile to ws[split][tile][256][256] (pgemm8_splitk_reduce sums)
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tail = gridDim.x / nsplit;
  const int t_local = b % tail, split = b / tail;
  const int nk_all = K / P8_BK;
  const int chunk = (nk_all + nsplit - 1) / nsplit;
  const int kbeg = split * chunk;
  const int nk = min(chunk, nk_all - kbeg);
  int tm, tn;
  p8_tile_mn(tile0 + t_local, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * P8_BM, n0 = tn * P8_BN;
  A += (int64_t)kbeg * P8_BK;
  W += (int64_t)kbeg * P8_BK;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases stay scalar
  const int wr = w >> 1, wc = w & 1;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, 0x7fffffff, 0x00020000);
  // DMA piece j of this wave: rows 64 w + 8 j + (lane >> 3); LDS slot lane & 7 <- chunk (lane & 7) ^ f(row)
  uint32_t va[8], vw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 64 * w + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    va[j] = m0 + row < M ? (uint32_t)((int64_t)(m0 + row) * lda + c * 16) : P8_OOB;
    const int wrow = EPI == P8_EPI_SILU_STD ? (row < 128 ? 0 : N / 2 - 128) + tn * 128 + row : n0 + row;
    vw[j] = (uint32_t)((int64_t)wrow * ldw + c * 16);
  }
  auto dma = [&](int kt, int j) {  // piece j < 8: A, j >= 8: W piece j - 8, K-step kt (clamped)
    const uint32_t so = (uint32_t)(min(kt, nk - 1) * P8_BK);
    char* dst = lds + (kt & 1) * P8_BUF + (j >= 8 ? P8_OPB : 0) + (8 * w + (j & 7)) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(j >= 8 ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             j >= 8 ? vw[j - 8] : va[j], so, 0, 0);
  };
  // fragment t (16 rows): row 16 t + (lane & 15), k 32 (lane >> 4) .. +31 = chunks 2q, 2q + 1
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fr >> 1) & 7;
  const int rd0 = fr * 128 + (((2 * fq) ^ sw) * 16), rd1 = fr * 128 + (((2 * fq + 1) ^ sw) * 16);
  const int a_rd = (wr * 128) * 128, w_rd = P8_OPB + (wc * 128) * 128;
  auto frag = [&](const char* buf, int base, int t) {
    const char* p = buf + base + t * 2048;
    const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(p + rd0);
    const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(p + rd1);
    return i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  const int one = 127;  // E8M0 1.0

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  i32x8_t fa[8], fw[2][8];

  // prologue: steps 0 and 1 in flight, step 0 landed, its W set and A fragments 0-6 in registers
#pragma unroll
  for (int j = 0; j < 16; ++j) dma(0, j);
#pragma unroll
  for (int j = 0; j < 16; ++j) dma(1, j);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  p8_bar();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    fw[0][j] = frag(lds, w_rd, j);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    fa[i] = frag(lds, a_rd, i);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // accumulator zero-init -> MFMA srcC
  __builtin_amdgcn_sched_barrier(0);

  // one K-step on W set S (the next step's W fragments go to set S ^ 1)
  auto step = [&](auto S_, int kt) {
    constexpr int S = decltype(S_)::value;
    const char* cur = lds + (kt & 1) * P8_BUF;
    const char* nxt = lds + ((kt & 1) ^ 1) * P8_BUF;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      mfma8(acc[i][j], fw[S][j], fa[i], one);
      if (t == 1) {
        fa[7] = frag(cur, a_rd, 7);
      } else if (t == 5) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's reads of the current buffer retired
        p8_bar();
      } else if (t >= 6 && t < 22) {
        dma(kt + 2, t - 6);
      } else if (t == 27) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step kt+1 landed (kt+2's 16 in flight)
        p8_bar();
      } else if (t >= 28 && t < 36) {
        fw[S ^ 1][t - 28] = frag(nxt, w_rd, t - 28);
      } else if (t >= 44 && t < 50) {
        fa[t - 44] = frag(nxt, a_rd, t - 44);
      } else if (t == 57) {
        fa[6] = frag(nxt, a_rd, 6);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // drain at the end of every step (asm MFMAs: hipcc does not model their latency)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(std::integral_constant<int, 0>{}, kt);
    step(std::integral_constant<int, 1>{}, kt + 1);
  }
  if (kt < nk) step(std::integral_constant<int, 0>{}, kt);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // ---- epilogue: acc[i][j][r] = C[m = 16 i + fr][n = 16 j + 4 fq + r] (wave-relative), x xs[m] ws[n]
  float sx[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + 16 * i + fr;
    sx[i] = m < M ? xs[m] : 0.f;
  }
  f32x4_t sn[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int nl = wc * 128 + 16 * j + 4 * fq;  // tile-relative column
    const int n = EPI == P8_EPI_SILU_STD ? (nl < 128 ? 0 : N / 2 - 128) + tn * 128 + nl : n0 + nl;
    sn[j] = *reinterpret_cast<const f32x4_t*>(wsc + n);
  }
  if constexpr (EPI == P8_EPI_F32) {
    float* wt = ws + ((int64_t)split * tail + t_local) * (P8_BM * P8_BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = wr * 128 + 16 * i + fr, col = wc * 128 + 16 * j + 4 * fq;
        const f32x4_t v = acc[i][j];
        *reinterpret_cast<f32x4_t*>(wt + row * P8_BN + col) =
            f32x4_t{v[0] * sx[i] * sn[j][0], v[1] * sx[i] * sn[j][1], v[2] * sx[i] * sn[j][2], v[3] * sx[i] * sn[j][3]};
      }
    return;
  }
  __syncthreads();
  char* img = lds + w * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 16 * i + fr, col = 16 * j + 4 * fq;
      const f32x4_t v = acc[i][j];
      u32x2_t p;
      p[0] = (uint32_t)f2bf(v[0] * sx[i] * sn[j][0]) | ((uint32_t)f2bf(v[1] * sx[i] * sn[j][1]) << 16);
      p[1] = (uint32_t)f2bf(v[2] * sx[i] * sn[j][2]) | ((uint32_t)f2bf(v[3] * sx[i] * sn[j][3]) << 16);
      *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
    }
  __syncthreads();
  if constexpr (EPI == P8_EPI_NONE) {
#pragma unroll 4
    for (int it = 0; it < 32; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int m = m0 + wr * 128 + row;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 + wc * 128 + c * 8) = v;
    }
  } else {
    // gate image of row-half wr: wave (wr, 0); up: wave (wr, 1); this wave stores 64 of its 128 rows
    const char* gimg = lds + (wr * 2) * 32768;
    const char* uimg = gimg + 32768;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int row = wc * 64 + it * 4 + (lane >> 4), c = lane & 15;
      const int m = m0 + wr * 128 + row;
      const int off = row * 256 + ((c ^ (row & 15)) * 16);
      float gf[8], uf[8], of[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(gimg + off), gf);
      unpack8(*reinterpret_cast<const u32x4_t*>(uimg + off), uf);
#pragma unroll
      for (int e = 0; e < 8; ++e) of[e] = gf[e] / (1.f + __expf(-gf[e])) * uf[e];
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + tn * 128 + c * 8) = pack8(of);
    }
  }
}

// sum of the nsplit scaled fp32 partials of tail tile t -> bf16 C (8 rows x 256 columns per block)
__global__ __launch_bounds__(256) void pgemm8_splitk_reduce(const float* __restrict__ ws, int nsplit, int tail,
                                                            int tile0, uint16_t* __restrict__ C, int64_t ldc, int M,
                                                            int N) {
  const int t = blockIdx.x / (P8_BM / 8), rblk = blockIdx.x % (P8_BM / 8);
  int tm, tn;
  p8_tile_mn(tile0 + t, (M + P8_BM - 1) / P8_BM, N / P8_BN, tm, tn);
  const int row = rblk * 8 + (threadIdx.x >> 5), col = (threadIdx.x & 31) * 8;
  const int m = tm * P8_BM + row;
  if (m >= M) return;
  float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float* src = ws + ((int64_t)s * tail + t) * (P8_BM * P8_BN) + row * P8_BN + col;
    const f32x4_t a = *reinterpret_cast<const f32x4_t*>(src);
    const f32x4_t b = *reinterpret_cast<const f32x4_t*>(src + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[e] += a[e];
      f[4 + e] += b[e];
    }
  }
  *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + tn * P8_BN + col) = pack8(f);
}

constexpr int P8_CUS = 256;  // MI355X compute units: one 256 x 256 tile per CU per wave

// tail split plan: a last wave at most half full, and a K long enough that each split keeps >= 8 steps
__host__ inline void pgemm8_plan(int M, int N, int K, int epi, int& full, int& tail, int& nsplit) {
  const int ntiles = ((M + P8_BM - 1) / P8_BM) * (N / P8_BN), nk = K / P8_BK;
  full = ntiles;
  tail = 0;
  nsplit = 1;
  const int t = ntiles % P8_CUS;
  if (epi != P8_EPI_NONE || t == 0 || 2 * t > P8_CUS) return;
  int s = std::min(P8_CUS / t, nk / 8);
  if (s < 2) return;
  full = ntiles - t;
  tail = t;
  nsplit = s;
}


// ---------------------------------------------------------------------------
// Persistent form (EPI_NONE): each workgroup walks tiles b, b + P, b + 2P, ... (P = min(#tiles,
// 256) workgroups) as ONE stream of K-steps g = 0 .. nt * nk - 1 with the schedule above, so the
// next tile's first two K-steps (and its 2 KB of scales) are DMA'd while the current tile's last
// steps compute - no per-tile prologue wait. The epilogue stores straight from the accumulators
// (both LDS buffers already hold the next tile): each lane writes 4 consecutive bf16 columns of a
// row (8 B); the tile's token / channel scales come from a small double-buffered LDS slot filled
// by the same LDS-DMA (a global load here would make hipcc wait vmcnt(0) on the DMAs in flight).
constexpr int P8_SCB = 2 * 256 * 4;             // one tile's xs (256 rows) + ws (256 columns)
constexpr int P8_LDS_P = 2 * P8_BUF + 2 * P8_SCB;

__global__ __launch_bounds__(P8_NT, 1) void pgemm8p_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ xs,
                                                           const uint8_t* __restrict__ W, int64_t ldw,
                                                           const float* __restrict__ wsc,
                                                           uint16_t* __restrict__ C, int64_t ldc, int M, int N,
                                                           int K, int ntiles) {
  __shared__ __attribute__((aligned(1024))) char lds[P8_LDS_P];  // the ONLY LDS object
  const int tiles_m = (M + P8_BM - 1) / P8_BM, tiles_n = N / P8_BN;
  const int P = gridDim.x;
  const int b = xcd_remap(blockIdx.x, P);
  const int nt = (ntiles - b + P - 1) / P;  // this workgroup's tiles: b, b + P, ...
  const int nk = K / P8_BK;
  const int S = nt * nk;                    // K-steps of this workgroup, all tiles

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rxs = __builtin_amdgcn_make_buffer_rsrc((void*)xs, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc((void*)wsc, 0, 0x7fffffff, 0x00020000);

  // DMA offsets of the tile being LOADED (two K-steps ahead of compute)
  uint32_t va[8], vw[8], vxs, vws;
  auto set_dma_tile = [&](int r) {
    int tm, tn;
    p8_tile_mn(b + min(r, nt - 1) * P, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 64 * w + 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      va[j] = tm * P8_BM + row < M ? (uint32_t)((int64_t)(tm * P8_BM + row) * lda + c * 16) : P8_OOB;
      vw[j] = (uint32_t)((int64_t)(tn * P8_BN + row) * ldw + c * 16);
    }
    const int m = tm * P8_BM + 64 * w + lane;
    vxs = m < M ? (uint32_t)(m * 4) : P8_OOB;
    vws = (uint32_t)((tn * P8_BN + 64 * w + lane) * 4);
  };
  // piece j (< 8: A, >= 8: W) of global step g, whose step within its tile is kt
  auto dma = [&](int g, int kt, int j) {
    char* dst = lds + (g & 1) * P8_BUF + (j >= 8 ? P8_OPB : 0) + (8 * w + (j & 7)) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(j >= 8 ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             j >= 8 ? vw[j - 8] : va[j], (uint32_t)(kt * P8_BK), 0, 0);
  };
  auto dma_scales = [&](int r) {  // tile r's scales into slot r & 1 (issued with its step-0 pieces)
    char* base = lds + 2 * P8_BUF + (r & 1) * P8_SCB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rxs, (__attribute__((address_space(3))) void*)(base + w * 256), 4, vxs,
                                             0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rws, (__attribute__((address_space(3))) void*)(base + 1024 + w * 256),
                                             4, vws, 0, 0, 0);
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fr >> 1) & 7;
  const int rd0 = fr * 128 + (((2 * fq) ^ sw) * 16), rd1 = fr * 128 + (((2 * fq + 1) ^ sw) * 16);
  const int a_rd = (wr * 128) * 128, w_rd = P8_OPB + (wc * 128) * 128;
  auto frag = [&](const char* buf, int base, int t) {
    const char* p = buf + base + t * 2048;
    const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(p + rd0);
    const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(p + rd1);
    return i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  const int one = 127;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  i32x8_t fa[8], fw[2][8];

  // prologue: global steps 0 and 1 (+ tile 0's scales) in flight, step 0 landed
  set_dma_tile(0);
  dma_scales(0);
#pragma unroll
  for (int j = 0; j < 16; ++j) dma(0, 0, j);
  if (nk == 1) set_dma_tile(1);
  if (nk == 1 && S > 1) dma_scales(1);
#pragma unroll
  for (int j = 0; j < 16; ++j) dma(1, nk == 1 ? 0 : 1, j);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  p8_bar();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    fw[0][j] = frag(lds, w_rd, j);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    fa[i] = frag(lds, a_rd, i);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // one K-step on W set SET; nk is even (host-checked), so every tile starts on set 0 and its
  // last step runs on set 1 (after which set 1 is dead: room for the epilogue's registers)
  auto step = [&](auto S_, int g, int kt) {
    constexpr int SET = decltype(S_)::value;
    const char* cur = lds + (g & 1) * P8_BUF;
    const char* nxt = lds + ((g & 1) ^ 1) * P8_BUF;
    const int g2 = g + 2;
    int kt2 = kt + 2;  // step of g + 2 within its tile (scalar bookkeeping, no division)
    if (kt2 >= nk) kt2 -= nk;
#pragma clang loop unroll(full)
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      mfma8(acc[i][j], fw[SET][j], fa[i], one);
      if (t == 1) {
        fa[7] = frag(cur, a_rd, 7);
      } else if (t == 5) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        p8_bar();
      } else if (t == 6) {
        if (kt2 == 0 && g2 < S) {  // g + 2 starts the next tile: its offsets and its scales
          set_dma_tile(g2 / nk);
          dma_scales(g2 / nk);
        }
        dma(g2, kt2, 0);
      } else if (t > 6 && t < 22) {
        dma(g2, kt2, t - 6);
      } else if (t == 27) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        p8_bar();
      } else if (t >= 28 && t < 36) {
        fw[SET ^ 1][t - 28] = frag(nxt, w_rd, t - 28);
      } else if (t >= 44 && t < 50) {
        fa[t - 44] = frag(nxt, a_rd, t - 44);
      } else if (t == 57) {
        fa[6] = frag(nxt, a_rd, 6);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int r = 0; r < nt; ++r) {
    for (int kt = 0; kt < nk; kt += 2) {
      const int g = r * nk + kt;
      step(std::integral_constant<int, 0>{}, g, kt);
      step(std::integral_constant<int, 1>{}, g + 1, kt + 1);
    }
    {  // tile r done: scale + store straight from the accumulators, then restart them
      int tm, tn;
      p8_tile_mn(b + r * P, tiles_m, tiles_n, tm, tn);
      const char* sb = lds + 2 * P8_BUF + (r & 1) * P8_SCB;
      const int mrow = tm * P8_BM + wr * 128 + fr;
      uint16_t* cb = C + (int64_t)tn * P8_BN + wc * 128 + 4 * fq;
#pragma unroll
      for (int i2 = 0; i2 < 8; ++i2) {
        const float sx = *reinterpret_cast<const float*>(sb + (wr * 128 + 16 * i2 + fr) * 4);
        const int m = mrow + 16 * i2;
#pragma unroll
        for (int j2 = 0; j2 < 8; ++j2) {
          const f32x4_t sn = *reinterpret_cast<const f32x4_t*>(sb + 1024 + (wc * 128 + 16 * j2 + 4 * fq) * 4);
          const f32x4_t v = acc[i2][j2];
          u32x2_t o;
          o[0] = (uint32_t)f2bf(v[0] * sx * sn[0]) | ((uint32_t)f2bf(v[1] * sx * sn[1]) << 16);
          o[1] = (uint32_t)f2bf(v[2] * sx * sn[2]) | ((uint32_t)f2bf(v[3] * sx * sn[3]) << 16);
          if (m < M) *reinterpret_cast<u32x2_t*>(cb + (int64_t)m * ldc + 16 * j2) = o;
        }
      }
#pragma unroll
      for (int i2 = 0; i2 < 8; ++i2)
#pragma unroll
        for (int j2 = 0; j2 < 8; ++j2) acc[i2][j2] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write -> MFMA srcC
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace

extern "C" int64_t llmd_pgemm_fp8_ws_bytes(int M, int N, int K, int epi) {
  if (M <= 0 || N % P8_BN || K % P8_BK) return 0;
  int full, tail, nsplit;
  pgemm8_plan(M, N, K, epi, full, tail, nsplit);
  return nsplit > 1 ? (int64_t)nsplit * tail * P8_BM * P8_BN * 4 : 0;
}

// epi 0: C [M, N]; epi 3: C [M, N / 2] = silu(gate) * up on W = [gate; up] ([N, K], N / 2 % 128 == 0)
extern "C" int llmd_pgemm_fp8(const void* A, int64_t lda, const float* xs, const void* W, int64_t ldw,
                              const float* ws, void* C, int64_t ldc, int M, int N, int K, int epi, void* wsp,
                              int persistent, hipStream_t st) {
  if (M <= 0) return 0;
  if (N % P8_BN || K % P8_BK || lda % 16 || ldw % 16 || ldc % 8) return -1;
  if (epi != P8_EPI_NONE && epi != P8_EPI_SILU_STD) return -3;
  if (epi == P8_EPI_SILU_STD && (N / 2) % 128) return -3;
  if ((int64_t)(M - 1) * lda + K > 0x7fffffffLL || (int64_t)(N - 1) * ldw + K > 0x7fffffffLL) return -2;
  int full = ((M + P8_BM - 1) / P8_BM) * (N / P8_BN), tail = 0, nsplit = 1;
  if (persistent && epi == P8_EPI_NONE) {
    if ((int64_t)M * 4 > 0x7fffffffLL || (K / P8_BK) % 2) return -2;
    hipLaunchKernelGGL(pgemm8p_kernel, dim3(std::min(full, P8_CUS)), dim3(P8_NT), 0, st, (const uint8_t*)A, lda, xs,
                       (const uint8_t*)W, ldw, ws, (uint16_t*)C, ldc, M, N, K, full);
    return (int)hipGetLastError();
  }
  if (wsp != nullptr) pgemm8_plan(M, N, K, epi, full, tail, nsplit);
  const auto* a = (const uint8_t*)A;
  const auto* w = (const uint8_t*)W;
  auto* c = (uint16_t*)C;
  if (epi == P8_EPI_SILU_STD)
    hipLaunchKernelGGL(pgemm8_kernel<P8_EPI_SILU_STD>, dim3(full), dim3(P8_NT), 0, st, a, lda, xs, w, ldw, ws, c,
                       ldc, M, N, K, 0, 1, nullptr);
  else if (full > 0)
    hipLaunchKernelGGL(pgemm8_kernel<P8_EPI_NONE>, dim3(full), dim3(P8_NT), 0, st, a, lda, xs, w, ldw, ws, c, ldc,
                       M, N, K, 0, 1, nullptr);
  if (nsplit > 1) {
    hipLaunchKernelGGL(pgemm8_kernel<P8_EPI_F32>, dim3(tail * nsplit), dim3(P8_NT), 0, st, a, lda, xs, w, ldw, ws, c,
                       ldc, M, N, K, full, nsplit, (float*)wsp);
    hipLaunchKernelGGL(pgemm8_splitk_reduce, dim3(tail * (P8_BM / 8)), dim3(256), 0, st, (const float*)wsp, nsplit,
                       tail, full, c, ldc, M, N);
  }
  return (int)hipGetLastError();
}
