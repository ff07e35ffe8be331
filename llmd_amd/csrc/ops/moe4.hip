// bf16 grouped expert GEMM v4 (prefill-sized MoE steps): the
// dense prefill GEMM's PGR2 structure (csrc/ops/pgemm.hip variant 3) on the
// 256-row expert tiles of moe_align(bm = 256).
//
//   Y[p, :] = X[row(p), :] . W[e(tile)]^T      p = a sorted slot of the tile
//
// One 256-thread workgroup per 256 x 256 tile (grid: N tiles x M tiles), 4
// waves x (128 x 128 of C) on v_mfma_f32_16x16x32_bf16 with AGPR accumulators.
// Each 64-deep K-step's fragments (both 32-deep halves) are read into
// registers before its LDS buffer is refilled, so two 64 KB buffers carry an
// LDS-DMA prefetch two K-steps deep (buffer_load ... lds: scalar buffer
// descriptors, 32-bit per-lane offsets, K offset in soffset). The A operand is
// GATHERED by the DMA itself: every lane's source offset points at its sorted
// slot's token row (padding slots read token 0 and are never stored), so no
// permuted copy of X exists. W rows past N (gpt-oss N = 5760 = 22.5 tiles) are
// clamped to row N - 1 and never stored.
//
// Epilogue through the then free LDS (per-wave [128][128] bf16 image, 16-B
// row stores): MODE 0 stores bf16 (+ per-expert bias); MODE 1 applies the
// gated activation on the interleaved [g0, u0, g1, u1, ..] N axis (SiLU, or
// gpt-oss clamped SwiGLU with alpha / limit) in registers - a lane holds 4
// consecutive columns, i.e. two (g, u) pairs - and stores N / 2 columns.
//
// Replaces the 8-wave v3 bf16 form (moe.hip moe_gemm3_fp8_kernel<.., BF>) for
// bf16 experts when ops.MOE_BF16_V4 is on (A/B: scripts/bench_moe.py).
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int M4_BM = 256, M4_BN = 256, M4_BK = 64, M4_NT = 256;
constexpr int M4_OPB = M4_BM * M4_BK * 2;  // 32 KB per operand per K-step
constexpr int M4_BUF = 2 * M4_OPB;         // 64 KB
constexpr int M4_RB = 37;                  // half-1 MFMA index of the next step's first read
// Per-lane DMA offset past the buffer descriptors' 0x7fffffff-byte range: the load is out of bounds
// and returns zeros. Padding slots and W rows past N (never stored) read it instead of a clamped
// real row, so their MFMAs multiply zeros: with the kernels at the 1400 W package cap, operand bits
// that do not toggle are clock (profiles/gemm_clock_power_r5.txt).
constexpr uint32_t M4_OOB = 0x80000000u;

__device__ __forceinline__ void m4_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void m4_mfma(f32x4_t& acc, const s16x8_t& a, const s16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ float m4_act(float g, float u, int act, float alpha, float limit) {
  if (act == 2) {  // gpt-oss: clamp, (u + 1) * g * sigmoid(alpha * g)
    g = fminf(g, limit);
    u = fminf(fmaxf(u, -limit), limit);
    return (u + 1.f) * g * __builtin_amdgcn_rcpf(1.f + __expf(-alpha * g));
  }
  return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)) * u;
}

// TBM: expert-tile rows, 256 or 192 (gpt-oss: ~160 rows per expert at a 5120-token step, so a
// 256-row tile is 62 % useful rows, a 192-row one 83 %). A wave owns TBM / 2 rows x 128 columns:
// MI = TBM / 32 A fragments of 16 rows; A DMA pieces per wave = MI, W pieces 8.
// (The 192 form first computed wrong rows from the second K-step on: hipcc had peeled the last
// iteration around a conditional drain and re-homed the accumulators right behind the loop's last
// asm MFMA - see the drain at the end of the K loop.)
template <int MODE, int TBM = 256>
__global__ __launch_bounds__(M4_NT, 1) void moe_gemm4_bf16_kernel(
    const uint16_t* __restrict__ X, int64_t x_stride, int topk, const int* __restrict__ sorted_ids,
    const int* __restrict__ tile_expert, const uint16_t* __restrict__ W, int64_t w_expert_stride, int N, int K,
    uint16_t* __restrict__ Y, int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots,
    const uint16_t* __restrict__ bias) {
  constexpr int MI = TBM / 32;             // 16-row A fragments per wave (8 / 6)
  constexpr int OPA = TBM * M4_BK * 2;     // A bytes per K-step
  constexpr int BUF = OPA + M4_OPB;        // A | W of one K-step
  constexpr int NPC = MI + 8;              // DMA pieces per wave per K-step (= fragment reads per half)
  constexpr int NMF = 8 * MI;              // MFMAs per half
  constexpr int TB = 8 * MI - 24;          // half 0: barrier MFMA index (A pieces of step kt + 2 after it)
  constexpr int WP = MI == 8 ? 5 : 4;      // half 1: one W piece every WP MFMAs
  constexpr int RB = MI == 8 ? M4_RB : 30; // half 1: first next-step read
  static_assert(TBM == 256 || TBM == 192, "tile rows");
  static_assert(TB + 1 + 3 * (MI - 1) < NMF && 8 + MI <= TB && 7 * WP < RB - 1 && RB + NPC <= NMF, "schedule");
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUF];  // the ONLY LDS object
  const int nt_ = blockIdx.x, mt = blockIdx.y;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * TBM, n0 = nt_ * M4_BN;
  const int nk = K / M4_BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W + (int64_t)e * w_expert_stride), 0, 0x7fffffff, 0x00020000);
  // DMA piece j: A rows 8 (MI w + j) + (lane >> 3), W rows 64 w + 8 j + (lane >> 3);
  // LDS slot lane & 7 <- chunk (lane & 7) ^ f(row)
  // fixed-size offset arrays: a template-dependent array size read by the DMA lambda makes hipcc's host
  // pass drop this kernel's launch stub (undefined symbol at load time)
  uint32_t va[8], vw[8];
#pragma unroll
  for (int j = 0; j < MI; ++j) {
    const int row = 8 * (MI * w + j) + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int sid = sorted_ids[m0 + row];
    const int tok = a_rows_are_slots ? m0 + row : sid / topk;
    va[j] = sid < 0 ? M4_OOB : (uint32_t)(((int64_t)tok * x_stride + c * 8) * 2);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 64 * w + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    vw[j] = n0 + row < N ? (uint32_t)(((int64_t)(n0 + row) * K + c * 8) * 2) : M4_OOB;
  }
  auto dma = [&](int kt, int j, bool wop) {
    const uint32_t so = (uint32_t)(min(kt, nk - 1) * M4_BK * 2);
    char* dst = lds + (kt & 1) * BUF + (wop ? OPA + (8 * w + j) * 1024 : (MI * w + j) * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wop ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             wop ? vw[j] : va[j], so, 0, 0);
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int rd0 = fr * 128 + ((fq ^ ((fr >> 1) & 7)) * 16);
  const int rd1 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) * 16);
  const int a_rd = (wr * (TBM / 2)) * 128, w_rd = OPA + (wc * 128) * 128;

  f32x4_t acc[MI][8];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s16x8_t fa0[MI], fw0[8], fa1[MI], fw1[8];

#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int j = 0; j < MI; ++j) dma(s2, j, false);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(s2, j, true);
  }
  if constexpr (NPC == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  m4_bar();
  fa0[0] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + rd0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fw0[i] = *reinterpret_cast<const s16x8_t*>(lds + w_rd + i * 2048 + rd0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 1; i < MI; ++i) {
    fa0[i] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + i * 2048 + rd0);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write (zero init) -> MFMA srcC
  __builtin_amdgcn_sched_barrier(0);

  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = lds + (kt & 1) * BUF;
    const char* nxt = lds + ((kt & 1) ^ 1) * BUF;
#pragma unroll
    for (int t = 0; t < NMF; ++t) {
      const int i = t >> 3, j = t & 7;
      // MFMA (0, j) needs the first j + 2 of this set's NPC reads, (1, 0) the first 10; the next
      // set's reads issued after MFMA 0 .. t - 1 are younger
      if (t <= 8) __builtin_amdgcn_s_waitcnt(0xC07F | ((NPC - 2) << 8));
      m4_mfma(acc[i][j], fw0[j], fa0[i]);
      if (t == 0) {
        fa1[0] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + rd1);
      } else if (t < 9) {
        fw1[t - 1] = *reinterpret_cast<const s16x8_t*>(cur + w_rd + (t - 1) * 2048 + rd1);
      } else if (t < 8 + MI) {
        fa1[t - 8] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (t - 8) * 2048 + rd1);
      } else if (t == TB) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        m4_bar();
      } else if (t > TB && (t - TB - 1) % 3 == 0 && (t - TB - 1) / 3 < MI) {
        dma(kt + 2, (t - TB - 1) / 3, false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < NMF; ++t) {
      const int i = t >> 3, j = t & 7;
      m4_mfma(acc[i][j], fw1[j], fa1[i]);
      if (t < 8 * WP && t % WP == 0) {
        dma(kt + 2, t / WP, true);
      } else if (t == RB - 1) {
        if constexpr (NPC == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        m4_bar();
      } else if (t == RB) {
        fa0[0] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + rd0);
      } else if (t > RB && t < RB + 9) {
        fw0[t - RB - 1] = *reinterpret_cast<const s16x8_t*>(nxt + w_rd + (t - RB - 1) * 2048 + rd0);
      } else if (t >= RB + 9 && t < RB + 8 + MI) {
        fa0[t - RB - 8] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (t - RB - 8) * 2048 + rd0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // drain the asm MFMAs at the end of EVERY iteration (~19 cycles of ~4000): hipcc cannot see
    // their latency, and accumulator copies can land right at the loop exit (epilogue spills). A
    // drain only in the last iteration made hipcc peel that iteration, with the accumulators
    // re-homed to other AGPRs by v_accvgpr_read / mov right behind the loop's last MFMA - stale
    // values (the 192-row form's wrong rows)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // asm MFMA results -> VALU reads
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: acc[i][j][r] = C[m][n], m = wr*TBM/2 + 16 i + (lane & 15), n = wc*128 + 16 j + 4 (lane >> 4) + r
  constexpr int WROWS = TBM / 2;
  char* img = lds + w * (WROWS * 256);
  const int ncol0 = n0 + wc * 128;
  // the expert bias of this lane's 8 x 4 columns, loaded once per tile (4 consecutive bf16 = one 8-B load;
  // N % 8 == 0 so a group is wholly in or out; columns past N are never stored)
  float bv[8][4];
  if (bias != nullptr) {
    const uint16_t* bp = bias + (int64_t)e * N;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = ncol0 + 16 * j + 4 * fq;
      const u32x2_t raw = n < N ? *reinterpret_cast<const u32x2_t*>(bp + n) : u32x2_t{0u, 0u};
      bv[j][0] = __uint_as_float(raw[0] << 16);
      bv[j][1] = __uint_as_float(raw[0] & 0xffff0000u);
      bv[j][2] = __uint_as_float(raw[1] << 16);
      bv[j][3] = __uint_as_float(raw[1] & 0xffff0000u);
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 16 * i + fr, col = 16 * j + 4 * fq;
      f32x4_t v = acc[i][j];
      if (bias != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bv[j][r];
      }
      if constexpr (MODE == 0) {
        u32x2_t p;
        p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
      } else {
        // two (g, u) pairs -> 2 outputs at half-columns col / 2, col / 2 + 1 of a [rows][64] image (128-B rows)
        const float o0 = m4_act(v[0], v[1], act, alpha, limit), o1 = m4_act(v[2], v[3], act, alpha, limit);
        const uint32_t p = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
        const int hc = col >> 1;  // 0..62, even
        *reinterpret_cast<uint32_t*>(img + row * 128 + (((hc >> 3) ^ (row & 7)) * 16) + (hc & 7) * 2) = p;
      }
    }
  __syncthreads();
  if constexpr (MODE == 0) {
#pragma unroll 4
    for (int it = 0; it < WROWS / 4; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int p = m0 + wr * WROWS + row;
      const int n = ncol0 + c * 8;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (sorted_ids[p] >= 0 && n < N) *reinterpret_cast<u32x4_t*>(Y + (int64_t)p * y_stride + n) = v;
    }
  } else {
#pragma unroll 4
    for (int it = 0; it < WROWS / 8; ++it) {
      const int row = it * 8 + (lane >> 3), c = lane & 7;
      const int p = m0 + wr * WROWS + row;
      const int n = ncol0 / 2 + c * 8;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 128 + ((c ^ (row & 7)) * 16));
      if (sorted_ids[p] >= 0 && 2 * n < N) *reinterpret_cast<u32x4_t*>(Y + (int64_t)p * y_stride + n) = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Block-scaled fp8 form (DeepGEMM role): e4m3 X [rows, Kp] with power-of-two
// per-(row, 128) scales xs, e4m3 W [E, N, Kp] with per-(128 x 128) scales ws
// [E, N / 128, Kp / 128]; v_mfma_scale_f32_32x32x64_f8f6f4 applies both as
// E8M0 exponents in hardware. A 64 KB K-step holds 128 fp8 of every row (the
// same 256 x 128-B images as the bf16 form), computed as 2 k-substeps of 4 x 4
// 32 x 32 x 64 MFMA per wave (64 cycles each: the step's 2048 MFMA cycles, with
// twice the bf16 FLOPs). The product is C^T (W fragments as the MFMA's A
// operand): the weight scale is one value per wave and K-step, the activation
// scale travels per lane (its token column), and a lane's accumulator holds 4
// consecutive N columns (one (g, u) pair per two). Activation scales ride the
// LDS-DMA (one 4-B piece per wave per step: 17 pieces, counted vmcnt(17)); the
// tile's weight scales are DMA'd once in the prologue.
typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void m8_mfma(f32x16_t& acc, const i32x8_t& a, const i32x8_t& b, int sa, int sb) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]"
               : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
}

// TBM 256 or 192 (as the bf16 form): a wave owns TBM / 2 rows = MB 32-row blocks (4 / 3); A DMA pieces
// per wave MB * 2 (8 / 6), act-scale piece: rows TBM / 4 * w + lane (clamped; 192: lanes 48-63 re-write
// the next wave's first rows with the same values).
template <int MODE, int TBM = 256>
__global__ __launch_bounds__(M4_NT, 1) void moe_gemm4_fp8_kernel(
    const uint8_t* __restrict__ X, int64_t x_stride, const float* __restrict__ xs, int64_t xs_stride, int topk,
    const int* __restrict__ sorted_ids, const int* __restrict__ tile_expert, const uint8_t* __restrict__ W,
    int64_t w_expert_stride, const float* __restrict__ ws, int N, int K, uint16_t* __restrict__ Y,
    int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots, const uint16_t* __restrict__ bias) {
  constexpr int MB = TBM / 64;                 // 32-row A blocks per wave
  constexpr int NA = 2 * MB;                   // A DMA pieces per wave per K-step
  constexpr int OPA = TBM * 128;               // A bytes per K-step (128 fp8 per row)
  constexpr int SCB = TBM * 4 + 256;           // act scales of a K-step (+ the 192 form's overhang)
  constexpr int BUF = OPA + M4_OPB + SCB;
  constexpr int WSO = 2 * BUF;                 // weight scales [2 col blocks][64 k-blocks]
  constexpr int LDSB = WSO + 2 * 64 * 4;
  constexpr int NPC = NA + 8 + 1;              // DMA pieces per wave per K-step (17 / 15)
  constexpr int NMF = 4 * MB;                  // MFMAs per k-substep
  constexpr int SROWS = TBM / 4;               // act-scale rows per wave
  static_assert(TBM == 256 || TBM == 192, "tile rows");
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];  // the ONLY LDS object
  const int nt_ = blockIdx.x, mt = blockIdx.y;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * TBM, n0 = nt_ * M4_BN;
  const int nk = K / 128, nnb = (N + 127) / 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int l32 = lane & 31, h = lane >> 5;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)xs, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W + (int64_t)e * w_expert_stride), 0, 0x7fffffff, 0x00020000);
  uint32_t va[8], vw[8];  // fixed size: see the bf16 form
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = 8 * (NA * w + j) + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int sid = sorted_ids[m0 + row];
    const int tok = a_rows_are_slots ? m0 + row : sid / topk;
    va[j] = sid < 0 ? M4_OOB : (uint32_t)((int64_t)tok * x_stride + c * 16);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 64 * w + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    vw[j] = n0 + row < N ? (uint32_t)((int64_t)(n0 + row) * K + c * 16) : M4_OOB;
  }
  uint32_t vs;  // this lane's act-scale row SROWS w + lane (clamped to the tile)
  {
    const int row = min(SROWS * w + lane, TBM - 1);
    const int sid = sorted_ids[m0 + row];
    const int tok = sid < 0 ? 0 : (a_rows_are_slots ? m0 + row : sid / topk);
    vs = (uint32_t)((int64_t)tok * xs_stride * 4);
  }
  auto dma = [&](int kt, int j, int op) {  // op 0 = A piece j, 1 = W piece j, 2 = act scales
    const int kc = min(kt, nk - 1);
    char* buf = lds + (kt & 1) * BUF;
    if (op == 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf + OPA + M4_OPB + w * SROWS * 4),
                                               4, vs, (uint32_t)(kc * 4), 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(op ? rw : ra,
                                               (__attribute__((address_space(3))) void*)(buf + (op ? OPA + (8 * w + j) * 1024 : (NA * w + j) * 1024)),
                                               16, op ? vw[j] : va[j], (uint32_t)(kc * 128), 0, 0);
  };
  // fragment of 32-row block b, k-substep s: lane row 32 b + l32, chunks 4 s + 2 h and 4 s + 2 h + 1
  auto frag = [&](const char* base, int b, int s) {
    const int row = 32 * b + l32;
    const int f = (row >> 1) & 7;
    const char* rp = base + row * 128;
    const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(rp + (((4 * s + 2 * h) ^ f) * 16));
    const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(rp + (((4 * s + 2 * h + 1) ^ f) * 16));
    return i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  const int a_base = wr * (TBM / 2) * 128, w_base = OPA + wc * 128 * 128;
  const int s_base = OPA + M4_OPB + wr * (TBM / 2) * 4;

  f32x16_t acc[4][MB];  // [W n-block j][A m-block i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < MB; ++i) acc[j][i] = f32x16_t{};
  i32x8_t fw0[4], fa0[MB], fw1[4], fa1[MB];
  int sa[MB];  // E8M0 act scales of this lane's token column in each m-block (current step)
  int swt;     // E8M0 weight scale of this wave's 128-column block (current step)
  float nsf[MB], nwf;  // the next step's raw scales

  // prologue: the tile's weight scales (waves 0 / 1: column blocks n0 / 128 + 0 / 1), steps 0 and 1
  if (w < 2) {
    const int cb = min(n0 / 128 + w, nnb - 1);
    const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(ws + ((int64_t)e * nnb + cb) * nk), 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rws, (__attribute__((address_space(3))) void*)(lds + WSO + w * 256), 4,
                                             (uint32_t)(min(lane, nk - 1) * 4), 0, 0, 0);
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int j = 0; j < NA; ++j) dma(s, j, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(s, j, 1);
    dma(s, 0, 2);
  }
  if constexpr (NPC == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");  // step 0 (and the weight scales) landed
  else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  m4_bar();
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    fw0[b] = frag(lds + w_base, b, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    fa0[b] = frag(lds + a_base, b, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) sa[b] = e8m0_of(*reinterpret_cast<const float*>(lds + s_base + (32 * b + l32) * 4));
  swt = e8m0_of(*reinterpret_cast<const float*>(lds + WSO + wc * 256));
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = lds + (kt & 1) * BUF;
    const char* nxt = lds + ((kt & 1) ^ 1) * BUF;
    // half 0 (k-substep 0): NMF MFMAs; reads of substep 1 (W then A) after the first 4 + MB; barrier
    // after them; A pieces (two per 64-cycle MFMA gap) + the act-scale piece of step kt + 2 to the end
#pragma unroll
    for (int t = 0; t < NMF; ++t) {
      const int j = t / MB, i = t % MB;
      m8_mfma(acc[j][i], fw0[j], fa0[i], swt, sa[i]);
      if (t < 4) {
        fw1[t] = frag(cur + w_base, t, 1);
      } else if (t < 4 + MB) {
        fa1[t - 4] = frag(cur + a_base, t - 4, 1);
      } else if (t == 4 + MB + 1) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        m4_bar();
      } else if (t > 4 + MB + 1 && t < 4 + MB + 2 + MB) {  // MB gaps x 2 A pieces
        const int q = t - (4 + MB + 2);
        dma(kt + 2, 2 * q, 0);
        dma(kt + 2, 2 * q + 1, 0);
        if (4 + 2 * MB + 2 >= NMF && t == NMF - 1) dma(kt + 2, 0, 2);  // 192 rows: the act-scale piece here
      } else if (t == 4 + 2 * MB + 2) {
        dma(kt + 2, 0, 2);  // the act-scale piece
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // half 1 (k-substep 1): W pieces of step kt + 2 after MFMA 0-7; step kt+1 landed + barrier after
    // MFMA 8; its substep-0 fragments and scales after
#pragma unroll
    for (int t = 0; t < NMF; ++t) {
      const int j = t / MB, i = t % MB;
      m8_mfma(acc[j][i], fw1[j], fa1[i], swt, sa[i]);
      if (t < 8) {
        dma(kt + 2, t, 1);
      } else if (t == 8) {
        if constexpr (NPC == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        m4_bar();
      } else if constexpr (MB == 4) {  // 16 MFMAs: one W fragment per gap, then A pairs
        if (t == 9) {  // the next step's raw scales, early (converted after the last MFMA)
#pragma unroll
          for (int b = 0; b < MB; ++b) nsf[b] = *reinterpret_cast<const float*>(nxt + s_base + (32 * b + l32) * 4);
          nwf = *reinterpret_cast<const float*>(lds + WSO + wc * 256 + min(kt + 1, nk - 1) * 4);
        }
        if (t >= 9 && t < 13) {
          fw0[t - 9] = frag(nxt + w_base, t - 9, 0);
        } else if (t >= 13 && t < 15) {
          fa0[2 * (t - 13)] = frag(nxt + a_base, 2 * (t - 13), 0);
          fa0[2 * (t - 13) + 1] = frag(nxt + a_base, 2 * (t - 13) + 1, 0);
        }
      } else {  // 12 MFMAs: the next set in the last three gaps
        if (t == 9) {
#pragma unroll
          for (int b = 0; b < MB; ++b) nsf[b] = *reinterpret_cast<const float*>(nxt + s_base + (32 * b + l32) * 4);
          nwf = *reinterpret_cast<const float*>(lds + WSO + wc * 256 + min(kt + 1, nk - 1) * 4);
          fw0[0] = frag(nxt + w_base, 0, 0);
          fw0[1] = frag(nxt + w_base, 1, 0);
        } else if (t == 10) {
          fw0[2] = frag(nxt + w_base, 2, 0);
          fw0[3] = frag(nxt + w_base, 3, 0);
        } else if (t == 11) {
#pragma unroll
          for (int b = 0; b < MB; ++b) fa0[b] = frag(nxt + a_base, b, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next step's scales (swapped in after this step's last MFMA used the current ones)
#pragma unroll
    for (int b = 0; b < MB; ++b) sa[b] = e8m0_of(nsf[b]);
    swt = e8m0_of(nwf);
    // drain at the end of every iteration (see the bf16 form): 16-pass MFMAs
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: acc[j][i][4 g + q] = C[m][n], m = wr*TBM/2 + 32 i + l32, n = wc*128 + 32 j + 8 g + 4 h + q
  constexpr int WROWS = TBM / 2;
  char* img = lds + w * (WROWS * 256);
  const int ncol0 = n0 + wc * 128;
  // the expert bias of this lane's 4 x 4 x 4 columns, loaded once per tile (one 8-B load per 4 columns)
  float bv[4][4][4];
  if (bias != nullptr) {
    const uint16_t* bp = bias + (int64_t)e * N;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = ncol0 + 32 * j + 8 * g + 4 * h;
        const u32x2_t raw = n < N ? *reinterpret_cast<const u32x2_t*>(bp + n) : u32x2_t{0u, 0u};
        bv[j][g][0] = __uint_as_float(raw[0] << 16);
        bv[j][g][1] = __uint_as_float(raw[0] & 0xffff0000u);
        bv[j][g][2] = __uint_as_float(raw[1] << 16);
        bv[j][g][3] = __uint_as_float(raw[1] & 0xffff0000u);
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = 32 * i + l32, col = 32 * j + 8 * g + 4 * h;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = acc[j][i][4 * g + q];
          if (bias != nullptr) v[q] += bv[j][g][q];
        }
        if constexpr (MODE == 0) {
          u32x2_t p;
          p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
        } else {
          const float o0 = m4_act(v[0], v[1], act, alpha, limit), o1 = m4_act(v[2], v[3], act, alpha, limit);
          const uint32_t p = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
          const int hc = col >> 1;
          *reinterpret_cast<uint32_t*>(img + row * 128 + (((hc >> 3) ^ (row & 7)) * 16) + (hc & 7) * 2) = p;
        }
      }
  __syncthreads();
  if constexpr (MODE == 0) {
#pragma unroll 4
    for (int it = 0; it < WROWS / 4; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int p = m0 + wr * WROWS + row;
      const int n = ncol0 + c * 8;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (sorted_ids[p] >= 0 && n < N) *reinterpret_cast<u32x4_t*>(Y + (int64_t)p * y_stride + n) = v;
    }
  } else {
#pragma unroll 4
    for (int it = 0; it < WROWS / 8; ++it) {
      const int row = it * 8 + (lane >> 3), c = lane & 7;
      const int p = m0 + wr * WROWS + row;
      const int n = ncol0 / 2 + c * 8;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 128 + ((c ^ (row & 7)) * 16));
      if (sorted_ids[p] >= 0 && 2 * n < N) *reinterpret_cast<u32x4_t*>(Y + (int64_t)p * y_stride + n) = v;
    }
  }
}

}  // namespace

extern "C" int llmd_moe_gemm4_bf16(const void* X, int64_t x_stride, int topk, const int* sorted_ids,
                                   const int* tile_expert, int num_tiles, const void* W, int64_t w_expert_stride,
                                   int N, int K, void* Y, int64_t y_stride, int mode, int act, float alpha,
                                   float limit, int a_rows_are_slots, const void* bias, int64_t x_rows, int tile_m,
                                   hipStream_t st) {
  if (K % M4_BK || x_stride % 8 || w_expert_stride % 8 || N % 8 || (mode == 1 && N % 16)) return -1;
  if (tile_m != 256 && tile_m != 192) return -1;
  // 31-bit byte offsets of the gathered rows and of one expert's weights
  if ((x_rows * x_stride + K) * 2 > 0x7fffffffLL || ((int64_t)N * K) * 2 > 0x7fffffffLL) return -2;
  if (num_tiles == 0) return 0;
  dim3 grid((N + M4_BN - 1) / M4_BN, num_tiles);
#define M4_LAUNCH(MODE_, TBM_)                                                                                    \
  hipLaunchKernelGGL((moe_gemm4_bf16_kernel<MODE_, TBM_>), grid, dim3(M4_NT), 0, st, (const uint16_t*)X, x_stride, \
                     topk, sorted_ids, tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y,        \
                     y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias)
  if (tile_m == 256) {
    if (mode == 0) M4_LAUNCH(0, 256); else M4_LAUNCH(1, 256);
  } else {
    if (mode == 0) M4_LAUNCH(0, 192); else M4_LAUNCH(1, 192);
  }
#undef M4_LAUNCH
  return (int)hipGetLastError();
}

extern "C" int llmd_moe_gemm4_fp8(const void* X, int64_t x_stride, const float* xs, int64_t xs_stride, int topk,
                                  const int* sorted_ids, const int* tile_expert, int num_tiles, const void* W,
                                  int64_t w_expert_stride, const float* ws, int N, int K, void* Y, int64_t y_stride,
                                  int mode, int act, float alpha, float limit, int a_rows_are_slots, const void* bias,
                                  int64_t x_rows, int tile_m, hipStream_t st) {
  // K: Kp (padded to 128), at most 64 k-blocks (the weight-scale row of a tile is one 64-lane DMA)
  if (K % 128 || K / 128 > 64 || x_stride % 16 || w_expert_stride % 16 || N % 8 || (mode == 1 && N % 16)) return -1;
  if (tile_m != 256 && tile_m != 192) return -1;
  if (x_rows * x_stride + K > 0x7fffffffLL || (int64_t)N * K > 0x7fffffffLL || x_rows * xs_stride * 4 > 0x7fffffffLL)
    return -2;
  if (num_tiles == 0) return 0;
  dim3 grid((N + M4_BN - 1) / M4_BN, num_tiles);
#define M8_LAUNCH(MODE_, TBM_)                                                                                    \
  hipLaunchKernelGGL((moe_gemm4_fp8_kernel<MODE_, TBM_>), grid, dim3(M4_NT), 0, st, (const uint8_t*)X, x_stride, xs, \
                     xs_stride, topk, sorted_ids, tile_expert, (const uint8_t*)W, w_expert_stride, ws, N, K,         \
                     (uint16_t*)Y, y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias)
  if (tile_m == 256) {
    if (mode == 0) M8_LAUNCH(0, 256); else M8_LAUNCH(1, 256);
  } else {
    if (mode == 0) M8_LAUNCH(0, 192); else M8_LAUNCH(1, 192);
  }
#undef M8_LAUNCH
  return (int)hipGetLastError();
}
