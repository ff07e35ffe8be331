// Prefill ("large-M") dense bf16 GEMM: C[M, N] = A[M, K] . W[N, K]^T, the
// QKV / O / gate-up / down projections of a prefill chunk (the
// hipBLASLt Cijk_* kernels that take ~68 % of the 70B serving bench).
//
// CDNA4 design (one 256 x 256 output tile per 512-thread workgroup, 1 per CU):
//   * 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 of C, as four 64 x 32
//     quadrants of 4 x 2 mfma_f32_16x16x32_bf16 tiles (128 accumulator regs);
//   * K-steps of 64 through TWO LDS buffers of 64 KB (A 256 x 128 B, W 256 x
//     128 B), each split into four 16 KB "halves" by the quadrant that reads
//     them (A: rows of quadrant-row 0 / 1, W: columns of quadrant-col 0 / 1).
//     A half is refilled by LDS-DMA (global_load_lds_dwordx4, no VGPR
//     staging) one phase after its last fragment read, so each K-step's loads
//     are in flight for ~6 phases, across the raw s_barriers, retired by
//     COUNTED vmcnt waits (never 0 inside the loop);
//   * 4 phases per K-step, one quadrant each (16 MFMA), fragment reads
//     front-loaded (12 / 4 / 8 / 0 ds_read_b128): both W halves stay in
//     registers for the whole K-step;
//   * waves 4-7 run one barrier behind waves 0-3 (stagger): on every SIMD one
//     wave's fragment reads + DMA issue overlap its partner's MFMA segment;
//   * 16-B chunks XOR-swizzled by (row & 7) on the DMA source address and on
//     the read (every ds_read_b128 lane group covers 16 distinct bank slots);
//   * XCD-aware tile order (each XCD walks its own contiguous range of tiles,
//     grouped 8 row-tiles deep so concurrently running tiles share A and W
//     panels in that XCD's L2);
//   * epilogue through the (then free) LDS: C is computed transposed (W frags
//     as the MFMA's first operand) so each lane holds 4 consecutive columns,
//     written as 8-B LDS stores, read back as 16-B rows and stored coalesced.
//     EPI_SILU: gate/up columns interleaved per 256-column tile (128 gate then
//     128 up, ops.pgemm_pack_gate_up) -> silu(g) * u is stored directly as the
//     [M, N/2] activation (no separate act kernel, no [M, N] round trip).
//
// Requirements (checked by the host wrapper): N % 256 == 0, K % 64 == 0,
// 16-B aligned rows; any M (rows past M are clamped on load, not stored).
#include <algorithm>
#include <type_traits>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int HALF = 16384;         // bytes of one half (128 rows x 128 B)
constexpr int BUF = 4 * HALF;       // one K-step: A q0, A q1, W q0, W q1
constexpr int LDS_BYTES = 2 * BUF;  // 128 KB
constexpr int GROUP_M = 8;

// EPI_SILU_STD (variants 3-5 only): the fused SiLU-and-mul on the model's own [gate; up] weight
// ([2F, K], F % 128 == 0): tile tn's W rows are gate rows [128 tn, +128) then up rows
// [F + 128 tn, +128) - the same tile image as EPI_SILU on a packed weight, no repacking.
enum { EPI_NONE = 0, EPI_SILU = 1, EPI_F32 = 2, EPI_SILU_STD = 3 };

__device__ __forceinline__ void dma16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

// wait until at most n (wave-uniform, 0..10) VMEM ops of this wave are outstanding
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// logical tile L (XCD-contiguous, GROUP_M-deep grouped order) -> (row tile, column tile)
__device__ __forceinline__ void tile_mn(int L, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GROUP_M * tiles_n;
  const int g = L / per_group, first_m = g * GROUP_M;
  const int gm = min(tiles_m - first_m, GROUP_M);
  tm = first_m + (L % per_group) % gm;
  tn = (L % per_group) / gm;
}

// Launch forms (host: llmd_pgemm, both variants): nsplit == 1 -> tiles [tile0, tile0 + grid)
// over the whole K (data-parallel); nsplit > 1 (EPI_F32) -> the grid covers `tail` tiles from
// tile0 x nsplit K-ranges, each block writing its fp32 partial tile to ws[split][tile][256][256]
// (pgemm_splitk_reduce sums them). The tail split turns a last, mostly idle wave of tiles
// (e.g. 576 tiles = 2.25 waves over 256 CUs at M 4608, N 8192) into one short full wave.
template <int EPI>
__global__ __launch_bounds__(NT, 1) void pgemm_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                      const uint16_t* __restrict__ W, int64_t ldw,
                                                      uint16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                      int tile0, int nsplit, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];  // the ONLY LDS object (see moe.hip G3)
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  // XCD-contiguous logical tile id, then GROUP_M-deep grouped order
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tail = gridDim.x / nsplit;
  const int t_local = b % tail, split = b / tail;
  const int nk_all = K / BK;
  const int chunk = (nk_all + nsplit - 1) / nsplit;
  const int kbeg = split * chunk;
  const int nk = min(chunk, nk_all - kbeg);
  int tm, tn;
  tile_mn(tile0 + t_local, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  A += (int64_t)kbeg * BK;
  W += (int64_t)kbeg * BK;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wr = w >> 2, wc = w & 3;

  // ---- DMA sources: half row i = 8 * (2w + j) + (lane >> 3), LDS chunk slot lane & 7
  // holds source chunk (lane & 7) ^ (i & 7); 32-bit element offsets from A / W
  uint32_t aoff[2][2], woff[2][2];  // [half][j]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 8 * (2 * w + j) + (lane >> 3);
      const int c = (lane & 7) ^ (i & 7);
      const int ar = min(m0 + (i >> 6) * 128 + h * 64 + (i & 63), M - 1);
      const int wn = n0 + (i >> 5) * 64 + h * 32 + (i & 31);
      aoff[h][j] = (uint32_t)(ar * lda + c * 8);
      woff[h][j] = (uint32_t)(wn * ldw + c * 8);
    }
  // half kinds in issue order: 0 = A q0, 1 = W q0, 2 = W q1, 3 = A q1; seq = 4 * ktile + kind
  auto issue = [&](int seq) {
    const int kt = seq >> 2, kind = seq & 3;
    char* dst = lds + (kt & 1) * BUF + (2 * w) * 1024;
    const int k0 = kt * BK;
    if (kind == 0 || kind == 3) {
      const int h = kind == 0 ? 0 : 1;
      dst += h * HALF;
      dma16(A + aoff[h][0] + k0, dst);
      dma16(A + aoff[h][1] + k0, dst + 1024);
    } else {
      const int h = kind - 1;
      dst += 2 * HALF + h * HALF;
      dma16(W + woff[h][0] + k0, dst);
      dma16(W + woff[h][1] + k0, dst + 1024);
    }
  };
  const int nseq = 4 * nk;
  int issued = 0;  // halves issued so far (wave-uniform)
  auto issue_upto = [&](int seq) {
    if (seq < nseq) {
      issue(seq);
      issued = seq + 1;
    }
  };
  // wait until half `seq` landed: 2 DMAs per younger half may stay in flight
  auto wait_seq = [&](int seq) { wait_vm(min(5, max(0, issued - seq - 1)) * 2); };

  // ---- fragment read offsets (bytes inside a half): lane row l & 15, chunk 4s + (l >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  int a_rd[4][2], w_rd[2][2];  // [mi][s], [ni][s]
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = wr * 64 + mi * 16 + fr;
      a_rd[mi][s] = i * 128 + (((4 * s + fq) ^ (i & 7)) * 16);
    }
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = wc * 32 + ni * 16 + fr;
      w_rd[ni][s] = i * 128 + (((4 * s + fq) ^ (i & 7)) * 16);
    }

  f32x4_t acc[2][2][4][2];  // [qm][qn][mi][ni]: C^T tiles (row = n, col = m)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  s16x8_t afr[4][2], wfr[2][2][2];  // [mi][s], [qn][ni][s]
  auto read_a = [&](const char* hb) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int s = 0; s < 2; ++s) afr[mi][s] = *reinterpret_cast<const s16x8_t*>(hb + a_rd[mi][s]);
  };
  auto read_w = [&](const char* hb, int qn) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int s = 0; s < 2; ++s) wfr[qn][ni][s] = *reinterpret_cast<const s16x8_t*>(hb + w_rd[ni][s]);
  };
  auto mfma_q = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[qm][qn][mi][ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[qn][ni][s], afr[mi][s], acc[qm][qn][mi][ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // one phase: [reads + DMA issue + counted wait] -> lgkmcnt(0) -> barrier -> MFMA -> barrier
  auto seg_end = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), visible to hipcc's waitcnt pass
    bar();
  };

  // ---- prologue: K-step 0 whole, K-step 1 but its A q1 half
#pragma unroll
  for (int s = 0; s < 7; ++s) issue_upto(s);
  wait_seq(1);
  bar();
  if (__builtin_amdgcn_readfirstlane(wr) == 1) bar();  // stagger: waves 4-7 one segment behind

  // one K-step: 4 phases of [fragment reads + DMA issue + counted wait] -> lgkmcnt(0) ->
  // barrier -> 16 MFMA -> barrier. STEADY (kt + 2 < nk): every refill exists and exactly
  // 5 younger halves (10 DMAs) stay in flight at each wait.
  auto ktile = [&](int kt, auto steady_t) {
    constexpr bool STEADY = decltype(steady_t)::value;
    const char* bufp = lds + (kt & 1) * BUF;
    // phase 1: A q0 + W q0 fragments; refill A q1 of K-step kt+1; W q1 (kt) lands for phase 2
    read_a(bufp);
    read_w(bufp + 2 * HALF, 0);
    if constexpr (STEADY) {
      issue(4 * (kt + 1) + 3);
      wait_vm(10);
    } else {
      issue_upto(4 * (kt + 1) + 3);
      wait_seq(4 * kt + 2);
    }
    seg_end();
    mfma_q(0, 0);
    bar();
    // phase 2: W q1 fragments; refill A q0 of kt+2 (its kt copy was read in phase 1)
    read_w(bufp + 3 * HALF, 1);
    if constexpr (STEADY) {
      issue(4 * (kt + 2) + 0);
      wait_vm(10);
    } else {
      issue_upto(4 * (kt + 2) + 0);
      wait_seq(4 * kt + 3);
    }
    seg_end();
    mfma_q(0, 1);
    bar();
    // phase 3: A q1 fragments; refill W q0 of kt+2
    read_a(bufp + HALF);
    if constexpr (STEADY) issue(4 * (kt + 2) + 1);
    else issue_upto(4 * (kt + 2) + 1);
    seg_end();
    mfma_q(1, 1);
    bar();
    // phase 4: no reads; refill W q1 of kt+2; A q0 + W q0 of kt+1 land for its phase 1
    if constexpr (STEADY) {
      issue(4 * (kt + 2) + 2);
      issued = 4 * (kt + 2) + 3;
      wait_vm(10);
    } else {
      issue_upto(4 * (kt + 2) + 2);
      if (kt + 1 < nk) wait_seq(4 * (kt + 1) + 1);
    }
    seg_end();
    mfma_q(1, 0);
    bar();
  };
  int kt = 0;
  for (; kt + 2 < nk; ++kt) ktile(kt, std::true_type{});
  for (; kt < nk; ++kt) ktile(kt, std::false_type{});
  if (__builtin_amdgcn_readfirstlane(wr) == 0) bar();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (EPI == EPI_F32) {
    float* wt = ws + ((int64_t)split * tail + t_local) * (BM * BN);
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            const int row = wr * 128 + qm * 64 + mi * 16 + (lane & 15);
            const int col = wc * 64 + qn * 32 + ni * 16 + (lane >> 4) * 4;
            *reinterpret_cast<f32x4_t*>(wt + row * BN + col) = acc[qm][qn][mi][ni];
          }
    return;
  }
  __syncthreads();

  // ---- epilogue: acc[qm][qn][mi][ni][r] = C[m][n] with
  //   m = wr*128 + qm*64 + mi*16 + (lane & 15), n = wc*64 + qn*32 + ni*16 + (lane >> 4)*4 + r
  // wave image in LDS: [128 rows (m)][64 cols (n)] bf16, 16-B chunks XOR-swizzled by row & 7
  char* img = lds + w * 16384;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const int row = qm * 64 + mi * 16 + fr;
          const int col = qn * 32 + ni * 16 + fq * 4;  // 4 consecutive bf16 = 8 B
          const f32x4_t v = acc[qm][qn][mi][ni];
          u32x2_t p;
          p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          const int chunk = (col >> 3) ^ (row & 7);
          *reinterpret_cast<u32x2_t*>(img + row * 128 + chunk * 16 + (col & 7) * 2) = p;
        }
  __syncthreads();
  if constexpr (EPI == EPI_NONE) {
    // each wave stores its own 128 x 64 block: 8 rows x 128 B per instruction
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int row = it * 8 + (lane >> 3), c = lane & 7;
      const int m = m0 + wr * 128 + row;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 128 + ((c ^ (row & 7)) * 16));
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 + wc * 64 + c * 8) = v;
    }
  } else {
    // EPI_SILU: tile columns [0,128) gate, [128,256) up -> 128 output columns at n0 / 2.
    // Waves wc = 0,1 hold gate cols [0,128), wc = 2,3 the matching up cols; the
    // wc < 2 waves combine their image with the partner wave's (wc + 2) image.
    if (wc < 2) {
      const char* up = lds + (w + 2) * 16384;
#pragma unroll 4
      for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3), c = lane & 7;
        const int m = m0 + wr * 128 + row;
        const int off = row * 128 + ((c ^ (row & 7)) * 16);
        float gf[8], uf[8], of[8];
        unpack8(*reinterpret_cast<const u32x4_t*>(img + off), gf);
        unpack8(*reinterpret_cast<const u32x4_t*>(up + off), uf);
#pragma unroll
        for (int e = 0; e < 8; ++e) of[e] = gf[e] / (1.f + __expf(-gf[e])) * uf[e];
        if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 / 2 + wc * 64 + c * 8) = pack8(of);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Variant 4W: 4 waves (one per SIMD), each 128 x 128 of C (8 x 8 tiles of
// mfma_f32_16x16x32_bf16: 256 accumulator registers, AGPR-resident), the form
// hipBLASLt's fastest MT256x256x64 kernels take. With one wave per SIMD the
// wave itself must keep its matrix pipe fed, so fragment reads are software-
// pipelined one k-substep (32) ahead in a second register set, interleaved
// 1 ds_read : 4 MFMA, and there are only two barriers per 64-deep K-step.
// LDS: 4 slots of 32 KB, slot (kt & 1) * 2 + h holds k-half h (32 wide) of
// K-step kt for A and W ([256 rows][64 B], 16-B chunks swizzled by
// F[(row >> 2) & 3], conflict-free for the 16x16x32 operand reads). A slot is
// refilled right after the barrier that follows its last fragment read, so
// every half has three substeps (~3000 cycles) to land; counted vmcnt(16).
constexpr int NT4 = 256;
constexpr int SLOT4 = 32768;  // one k-half of A (16 KB) + of W (16 KB)

// The 64 accumulators (256 registers) fill the accumulator file exactly; through the
// builtin, hipcc's register allocator re-homes loop-carried accumulators every
// iteration (~100-450 v_accvgpr moves per 64 MFMAs, with MFMA-result read stalls).
// As an asm statement with the accumulator TIED in an AGPR ("+a") every tile stays
// in place (0 moves). Hazards the compiler cannot see: an MFMA result read by a
// non-MFMA instruction needs 12 wait states (8-pass XDL) -> mfma_drain() before the
// epilogue; the A/B operands come straight from ds_read (lgkmcnt-ordered by hipcc,
// which tracks the asm's "v" inputs), never from a VALU write in the 2 states before.
__device__ __forceinline__ void mfma16_acc(f32x4_t& acc, const s16x8_t& a, const s16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7" ::: "memory"); }

__device__ __forceinline__ int swz4(int row, int c) {
  // F = {0, 2, 3, 1}: every ds_read_b128 lane group of a 16 x 4-chunk read hits 16 distinct slots
  return c ^ ((0x1E >> (2 * ((row >> 2) & 3))) & 3);
}

// Same launch forms as pgemm_kernel (tile0 / nsplit / ws).
template <int EPI>
__global__ __launch_bounds__(NT4, 1) void pgemm4_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                        const uint16_t* __restrict__ W, int64_t ldw,
                                                        uint16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        int tile0, int nsplit, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(1024))) char lds[4 * SLOT4];  // the ONLY LDS object
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tail = gridDim.x / nsplit;
  const int t_local = b % tail, split = b / tail;
  const int nk_all = K / BK;
  const int chunk = (nk_all + nsplit - 1) / nsplit;
  const int kbeg = split * chunk;
  const int nk = min(chunk, nk_all - kbeg);
  int tm, tn;
  tile_mn(tile0 + t_local, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  A += (int64_t)kbeg * BK;
  W += (int64_t)kbeg * BK;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wr = w >> 1, wc = w & 1;

  // DMA: a k-half of A is 256 rows x 64 B = 16 pieces of 1 KB (16 rows each); wave w moves
  // pieces 4w..4w+3 of A and of W. Lane: row 16 * piece + (lane >> 2), slot lane & 3.
  uint32_t aoff[4], woff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 16 * (4 * w + j) + (lane >> 2);
    const int c = swz4(row, lane & 3);
    aoff[j] = (uint32_t)(min(m0 + row, M - 1) * lda + c * 8);
    woff[j] = (uint32_t)((n0 + row) * ldw + c * 8);
  }
  // half index q = 2 * kt + h, slot (kt & 1) * 2 + h = q & 3; a half is 8 LDS-DMA pieces per wave
  // (A rows 0..3, W rows 4..7)
  auto issue_piece = [&](int q, int p) {
    char* dst = lds + (q & 3) * SLOT4 + (4 * w) * 1024;
    const int k0 = (q >> 1) * BK + (q & 1) * 32;
    if (p < 4) dma16(A + aoff[p] + k0, dst + p * 1024);
    else dma16(W + woff[p - 4] + k0, dst + 16384 + (p - 4) * 1024);
  };
  auto issue = [&](int q) {
#pragma unroll
    for (int p = 0; p < 8; ++p) issue_piece(q, p);
  };
  const int nq = 2 * nk;

  // fragment reads: tile row r = 16 * t + (lane & 15), chunk lane >> 4; (r >> 2) & 3 does not depend on t
  const int fr = lane & 15, fq = lane >> 4;
  const int rd = fr * 64 + swz4(fr, fq) * 16;
  const int a_rd = (wr * 128) * 64 + rd, w_rd = 16384 + (wc * 128) * 64 + rd;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s16x8_t fa0[8], fw0[8], fa1[8], fw1[8];
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write (zero init) -> MFMA srcC
  __builtin_amdgcn_sched_barrier(0);

  // One substep = 64 MFMAs on (fa, fw), row i of 8 at a time. Around each row: the next
  // substep's two fragment reads of row i (from `nxt` into na / nw) before it, and one of
  // the 8 LDS-DMA pieces of half `dq` (the refill of the slot the PREVIOUS substep read)
  // after it - DMA issue costs ~60-180 cycles each, so it must ride inside the MFMA stream,
  // not stall the wave at the boundary.
#define PG4_SUBSTEP(fa, fw, na, nw, nxt, dq)                                                               \
  {                                                                                                        \
    const char* nb_ = (nxt);                                                                               \
    const bool dma_ = (dq) < nq;                                                                           \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                        \
      na[i] = *reinterpret_cast<const s16x8_t*>(nb_ + a_rd + i * 1024);                                    \
      nw[i] = *reinterpret_cast<const s16x8_t*>(nb_ + w_rd + i * 1024);                                    \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) mfma16_acc(acc[i][j], fw[j], fa[i]);                   \
      if (dma_) issue_piece((dq), i);                                                                      \
      __builtin_amdgcn_sched_barrier(0);                                                                   \
    }                                                                                                      \
  }
  // boundary: this wave's fragment reads retired, the half read next has landed (every wave,
  // after the barrier)
  auto boundary = [&](int wait_q, int issued_hi) {
    // lgkmcnt(0) as the builtin, so hipcc's waitcnt pass sees the fragment reads retired
    // (after an asm wait it re-waits before the next substep's first MFMA)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const int younger = min(2, max(0, issued_hi - wait_q - 1));
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
  };

  // prologue: halves 0..3 (K-steps 0, 1); read K-step 0 half 0 fragments
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nq) issue(q);
  {
    const int hi = min(4, nq);
    const int younger = hi - 1;  // wait for half 0
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa0[i] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + i * 1024);
    fw0[i] = *reinterpret_cast<const s16x8_t*>(lds + w_rd + i * 1024);
  }
  // before half 1 of K-step 0 is read (during substep (0, 0)) it must have landed
  {
    const int hi = min(4, nq);
    const int younger = hi - 2;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // the prologue fragments, visibly to hipcc (else it re-waits in the loop)
    bar();
  }
  int issued = min(4, nq);
  // Substep u = 2 kt + s computes half u, reads half u + 1 and refills with half u + 4 the
  // slot of half u (read by substep u - 1, retired by the boundary before u). Every K-step
  // in one loop body (a peeled last step makes hipcc re-home the accumulators): the last
  // step's read-ahead of the nonexistent next half reads a stale slot into registers nothing
  // consumes, its waits drain to 0.
  for (int kt = 0; kt < nk; ++kt) {
    const int q0 = 2 * kt;
    PG4_SUBSTEP(fa0, fw0, fa1, fw1, lds + ((q0 + 1) & 3) * SLOT4, q0 + 4);
    if (q0 + 4 < nq) issued = q0 + 5;
    boundary(q0 + 2, issued);
    PG4_SUBSTEP(fa1, fw1, fa0, fw0, lds + ((q0 + 2) & 3) * SLOT4, q0 + 5);
    if (q0 + 5 < nq) issued = q0 + 6;
    boundary(q0 + 3, issued);
  }
#undef PG4_SUBSTEP
  mfma_drain();  // the last MFMA results before the epilogue reads them (asm MFMAs are opaque to hipcc)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (EPI == EPI_F32) {
    // fp32 partial tile, row-major [256][256]: 4 consecutive columns per lane -> 16-B stores
    float* wt = ws + ((int64_t)split * tail + t_local) * (BM * BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = wr * 128 + 16 * i + fr, col = wc * 128 + 16 * j + 4 * fq;
        *reinterpret_cast<f32x4_t*>(wt + row * BN + col) = acc[i][j];
      }
    return;
  }
  __syncthreads();

  // epilogue: acc[i][j][r] = C[m][n], m = wr*128 + 16 i + (lane & 15), n = wc*128 + 16 j + 4 (lane >> 4) + r.
  // wave image: [128 rows][128 cols] bf16 (256-B rows), 16-B chunks XOR-swizzled by row & 15
  char* img = lds + w * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 16 * i + fr, col = 16 * j + 4 * fq;
      const f32x4_t v = acc[i][j];
      u32x2_t p;
      p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
    }
  __syncthreads();
  if constexpr (EPI == EPI_NONE) {
#pragma unroll 4
    for (int it = 0; it < 32; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int m = m0 + wr * 128 + row;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 + wc * 128 + c * 8) = v;
    }
  } else {
    // gate = tile columns [0, 128) (waves wc = 0), up = [128, 256) (wc = 1): wave (wr, 0) combines
    if (wc == 0) {
      const char* up = lds + (w + 1) * 32768;
#pragma unroll 4
      for (int it = 0; it < 32; ++it) {
        const int row = it * 4 + (lane >> 4), c = lane & 15;
        const int m = m0 + wr * 128 + row;
        const int off = row * 256 + ((c ^ (row & 15)) * 16);
        float gf[8], uf[8], of[8];
        unpack8(*reinterpret_cast<const u32x4_t*>(img + off), gf);
        unpack8(*reinterpret_cast<const u32x4_t*>(up + off), uf);
#pragma unroll
        for (int e = 0; e < 8; ++e) of[e] = gf[e] / (1.f + __expf(-gf[e])) * uf[e];
        if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 / 2 + c * 8) = pack8(of);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Variant 2 ("RS4"): the 4-wave / 128 x 128-per-wave form of variant 1, but the
// operands are REGISTER-staged (global_load_dwordx4 -> VGPR -> ds_write_b128)
// instead of LDS-DMA. Why: with one wave per SIMD there is no partner wave to
// hide an instruction's issue cost behind, and an LDS-DMA piece costs ~60-180
// cycles of issue among MFMAs (MI355X_MICROARCH.md, LDS-DMA piece row) - 8 per
// 64 MFMA (1024 cycles) in variant 1 - while a global_load / ds_write issues in
// a few cycles. One wave per SIMD has 512 registers (256 AGPR accumulators +
// 256 VGPR), so the staging ring that would not fit at two waves per SIMD fits.
//
// Per 64-deep K-step kt (LDS buffer cur = kt & 1, 2 x 64 KB):
//   substep 0: 64 MFMA on fragment set 0 (k 0..31); between MFMA rows: the 16
//              fragment reads of set 1 (k 32..63) from buf cur and the 16
//              ds_write_b128 of step kt+1's staged tile into buf cur ^ 1;
//   lgkmcnt(0) + s_barrier (the ONE barrier per K-step);
//   substep 1: 64 MFMA on set 1; between rows: the 16 fragment reads of step
//              kt+1's set 0 from buf cur ^ 1 and the 16 global loads of step
//              kt+2 into the staging registers.
// Buffer cur ^ 1 was last read in step kt-1's substep 0, before step kt-1's
// barrier, so substep 0 of kt may overwrite it; it is read again only after
// step kt's barrier. W fragments are read before A fragments in each set (every
// MFMA row needs all 8 W fragments). LDS image: [256 rows][64 k] bf16 per
// operand, 16-B chunk c of row r at chunk c ^ ((r >> 1) & 7): conflict-free for
// the ds_read_b128 lane groups of the 16 x 16 x 32 operand reads and for the
// 8-lane ds_write_b128 groups (one 128-B row each).
constexpr int NT5 = 256;
constexpr int OPB5 = BM * BK * 2;  // one operand of one K-step: 32 KB
constexpr int BUF5 = 2 * OPB5;     // A + W

__device__ __forceinline__ int swz5(int row, int c) { return c ^ ((row >> 1) & 7); }

template <int EPI>
__global__ __launch_bounds__(NT5, 1) void pgemm5_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                        const uint16_t* __restrict__ W, int64_t ldw,
                                                        uint16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        int tile0, int nsplit, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUF5];  // the ONLY LDS object
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tail = gridDim.x / nsplit;
  const int t_local = b % tail, split = b / tail;
  const int nk_all = K / BK;
  const int chunk = (nk_all + nsplit - 1) / nsplit;
  const int kbeg = split * chunk;
  const int nk = min(chunk, nk_all - kbeg);
  int tm, tn;
  tile_mn(tile0 + t_local, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  A += (int64_t)kbeg * BK;
  W += (int64_t)kbeg * BK;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wr = w >> 1, wc = w & 1;

  // staging: load i (0..7) of an operand = row 32 i + (tid >> 3), chunk tid & 7
  const int srow = tid >> 3, sc = tid & 7;
  uint32_t aoff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) aoff[i] = (uint32_t)(min(m0 + 32 * i + srow, M - 1) * lda + sc * 8);
  const uint32_t woff0 = (uint32_t)((n0 + srow) * ldw + sc * 8);
  const uint32_t wstep = (uint32_t)(32 * ldw);
  // LDS byte offset of this thread's chunk in row 32 i + srow ((32 i + srow) >> 1 & 7 == (srow >> 1) & 7)
  const int st_off = srow * 128 + swz5(srow, sc) * 16;

  // fragment reads: row 16 t + (lane & 15), chunk 4 s + (lane >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  const int rd0 = fr * 128 + swz5(fr, fq) * 16, rd1 = fr * 128 + swz5(fr, 4 + fq) * 16;
  const int a_rd = (wr * 128) * 128, w_rd = OPB5 + (wc * 128) * 128;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s16x8_t fa0[8], fw0[8], fa1[8], fw1[8];
  u32x4_t ga[8], gw[8];

  auto gload = [&](int kt, int i) {  // loads i of A and of W, K-step kt
    const int k0 = min(kt, nk - 1) * BK;
    ga[i] = *reinterpret_cast<const u32x4_t*>(A + aoff[i] + k0);
    gw[i] = *reinterpret_cast<const u32x4_t*>(W + woff0 + i * wstep + k0);
  };
  auto swrite = [&](char* buf, int i) {
    *reinterpret_cast<u32x4_t*>(buf + i * 4096 + st_off) = ga[i];
    *reinterpret_cast<u32x4_t*>(buf + OPB5 + i * 4096 + st_off) = gw[i];
  };

  // prologue: step 0 -> buf 0, step 1 -> staging, set 0 of step 0 -> registers
#pragma unroll
  for (int i = 0; i < 8; ++i) gload(0, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) swrite(lds, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) gload(1, i);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's ds_writes done
  bar();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fw0[i] = *reinterpret_cast<const s16x8_t*>(lds + w_rd + i * 2048 + rd0);
    fa0[i] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + i * 2048 + rd0);
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write (zero init) -> MFMA srcC
  __builtin_amdgcn_sched_barrier(0);

  // one MFMA row i (8 MFMA on acc[i][*]) with two "side" instructions after it
#define PG5_ROW(fa, fw, i, SIDE)                                                       \
  {                                                                                    \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) mfma16_acc(acc[i][j], fw[j], fa[i]); \
    SIDE;                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = lds + (kt & 1) * BUF5;
    char* nxt = lds + ((kt & 1) ^ 1) * BUF5;
    // substep 0: set 0; read set 1 (W first) from cur, write step kt+1 into nxt
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      PG5_ROW(fa0, fw0, i, {
        if (i < 4) {
          fw1[2 * i] = *reinterpret_cast<const s16x8_t*>(cur + w_rd + (2 * i) * 2048 + rd1);
          fw1[2 * i + 1] = *reinterpret_cast<const s16x8_t*>(cur + w_rd + (2 * i + 1) * 2048 + rd1);
        } else {
          fa1[2 * i - 8] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (2 * i - 8) * 2048 + rd1);
          fa1[2 * i - 7] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (2 * i - 7) * 2048 + rd1);
        }
        swrite(nxt, i);
      });
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): set-1 reads and the nxt writes retired
    bar();
    // substep 1: set 1; read step kt+1's set 0 (W first) from nxt, load step kt+2
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      PG5_ROW(fa1, fw1, i, {
        if (i < 4) {
          fw0[2 * i] = *reinterpret_cast<const s16x8_t*>(nxt + w_rd + (2 * i) * 2048 + rd0);
          fw0[2 * i + 1] = *reinterpret_cast<const s16x8_t*>(nxt + w_rd + (2 * i + 1) * 2048 + rd0);
        } else {
          fa0[2 * i - 8] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (2 * i - 8) * 2048 + rd0);
          fa0[2 * i - 7] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (2 * i - 7) * 2048 + rd0);
        }
        gload(kt + 2, i);
      });
    }
  }
#undef PG5_ROW
  mfma_drain();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (EPI == EPI_F32) {
    float* wt = ws + ((int64_t)split * tail + t_local) * (BM * BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = wr * 128 + 16 * i + fr, col = wc * 128 + 16 * j + 4 * fq;
        *reinterpret_cast<f32x4_t*>(wt + row * BN + col) = acc[i][j];
      }
    return;
  }
  __syncthreads();
  // epilogue (as variant 1): acc[i][j][r] = C[m][n], m = wr*128 + 16 i + (lane & 15),
  // n = wc*128 + 16 j + 4 (lane >> 4) + r; per-wave [128][128] bf16 image, chunks XOR row & 15
  char* img = lds + w * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 16 * i + fr, col = 16 * j + 4 * fq;
      const f32x4_t v = acc[i][j];
      u32x2_t p;
      p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
    }
  __syncthreads();
  if constexpr (EPI == EPI_NONE) {
#pragma unroll 4
    for (int it = 0; it < 32; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int m = m0 + wr * 128 + row;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 + wc * 128 + c * 8) = v;
    }
  } else {
    // gate = tile columns [0, 128) (waves wc = 0), up = [128, 256) (wc = 1): both waves of a row
    // half store 64 rows each of silu(g) * u
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
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 / 2 + c * 8) = pack8(of);
    }
  }
}

// ---------------------------------------------------------------------------
// Variant 3 ("PGR2"): 4 waves x (128 x 128 of C) as variant 1, restructured so
// that each 64-deep K-step's fragments (both 32-deep halves, 32 ds_read_b128 =
// 128 VGPR) are read into registers BEFORE its LDS buffer is refilled. With the
// whole step register-resident, two 64 KB LDS buffers carry a global prefetch
// two K-steps deep (step kt+2 streams into the buffer step kt was read from),
// so every LDS-DMA piece has ~1.5 K-steps (~3000 cycles) to land.
//
// Per K-step kt (buffer b = kt & 1), 128 MFMA in two halves of 64:
//   half 0 (set 0, k 0..31): MFMA 0-15 each followed by one ds_read of set 1
//     (k 32..63 of step kt, W fragments first); at MFMA 40 lgkmcnt(0) +
//     barrier (every wave has read ALL of buffer b); MFMA 41-63 carry the 8
//     A-tile LDS-DMA pieces of step kt+2 into buffer b, one per 3 MFMA;
//   half 1 (set 1): MFMA 0-35 carry the 8 W-tile pieces (one per 5 MFMA); at
//     MFMA 36 vmcnt(16) (step kt+1's pieces, issued one K-step ago, landed;
//     this step's 16 stay in flight) + barrier; MFMA 37-52 each followed by one
//     ds_read of step kt+1's set 0 from buffer b ^ 1 (11 MFMA of slack before
//     the next step's first MFMA needs them).
// LDS-DMA through buffer_load_dwordx4 ... lds: one scalar buffer descriptor per
// operand, a 32-bit per-lane offset fixed for the whole loop, the K offset in
// soffset and the LDS base in m0 - a handful of scalar instructions per piece,
// no per-piece 64-bit address math, no branch (the step index is clamped; the
// two surplus steps at the end reload the last tile into a buffer nobody reads).
// LDS image per operand: [256 rows][64 k] bf16, each 1 KB DMA piece = 8 rows;
// 16-B chunk c of row r sits at slot c ^ ((r >> 1) & 7) (source-side swizzle,
// conflict-free for the 16 x 16 x 32 operand reads).
constexpr int NT6 = 256;
// RB6: half-1 MFMA index of the first read of the next step (its barrier one before);
// AUX6: cache-policy bits of the LDS-DMA loads (0, or 16 = sc1 as hipBLASLt's kernels use)
constexpr int OPB6 = BM * BK * 2;  // 32 KB per operand per K-step
constexpr int BUF6 = 2 * OPB6;     // 64 KB

template <int EPI, int RB6 = 37, int AUX6 = 0>
__global__ __launch_bounds__(NT6, 1) void pgemm6_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                        const uint16_t* __restrict__ W, int64_t ldw,
                                                        uint16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        int tile0, int nsplit, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUF6];  // the ONLY LDS object
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tail = gridDim.x / nsplit;
  const int t_local = b % tail, split = b / tail;
  const int nk_all = K / BK;
  const int chunk = (nk_all + nsplit - 1) / nsplit;
  const int kbeg = split * chunk;
  const int nk = min(chunk, nk_all - kbeg);
  int tm, tn;
  tile_mn(tile0 + t_local, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases stay scalar
  const int wr = w >> 1, wc = w & 1;

  // buffer descriptors over the K-range of this split (byte offsets must fit 31 bits: host-checked)
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)kbeg * BK), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)kbeg * BK), 0, 0x7fffffff, 0x00020000);
  // DMA piece j of this wave: rows 64 w + 8 j + (lane >> 3), LDS slot lane & 7 <- chunk (lane & 7) ^ f(row)
  uint32_t va[8], vw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 64 * w + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    va[j] = m0 + row < M ? (uint32_t)(((m0 + row) * lda + c * 8) * 2) : 0x80000000u;  // past M: OOB zeros
    const int wrow = EPI == EPI_SILU_STD ? (row < 128 ? 0 : N / 2 - 128) + tn * 128 + row : n0 + row;
    vw[j] = (uint32_t)((wrow * ldw + c * 8) * 2);
  }
  auto dma = [&](int kt, int j, bool wop) {  // piece j of operand A (wop = false) or W, K-step kt
    const uint32_t so = (uint32_t)(min(kt, nk - 1) * BK * 2);
    char* dst = lds + (kt & 1) * BUF6 + (wop ? OPB6 : 0) + (8 * w + j) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wop ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             wop ? vw[j] : va[j], so, 0, AUX6);
  };

  // fragment reads: row 16 t + (lane & 15), chunk 4 h + (lane >> 4) at slot chunk ^ ((lane >> 1) & 7)
  const int fr = lane & 15, fq = lane >> 4;
  const int rd0 = fr * 128 + ((fq ^ ((fr >> 1) & 7)) * 16);
  const int rd1 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) * 16);
  const int a_rd = (wr * 128) * 128, w_rd = OPB6 + (wc * 128) * 128;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s16x8_t fa0[8], fw0[8], fa1[8], fw1[8];

  // prologue: steps 0 and 1 in flight, step 0 landed, its set 0 in registers
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, j, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, j, true);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, j, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, j, true);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  bar();
  // read order of a set (everywhere): A row 0, the 8 W fragments, A rows 1..7 - MFMA (0, j) then
  // needs only the first j + 2 reads, so the waits before the first MFMA row are progressive
  fa0[0] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + rd0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fw0[i] = *reinterpret_cast<const s16x8_t*>(lds + w_rd + i * 2048 + rd0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    fa0[i] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + i * 2048 + rd0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // nothing pending on the loop's entry edge: hipcc's waitcnt pass then keeps the counted
  // waits of the back edge at the loop head instead of merging to lgkmcnt(0) every K-step
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write (zero init) -> MFMA srcC
  __builtin_amdgcn_sched_barrier(0);

  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = lds + (kt & 1) * BUF6;
    const char* nxt = lds + ((kt & 1) ^ 1) * BUF6;
    // ---- half 0: set 0; reads of set 1; barrier; A pieces of step kt + 2
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      // explicit progressive waits for set 0 (hipcc's own pass waits lgkmcnt(0) at the loop head):
      // MFMA (0, j) needs the first j + 2 of set 0's 16 reads, (i, 0) the first i + 9; the set-1
      // reads issued after MFMA 0 .. t - 1 are younger still
      // (row 1: 7 - 1 + 8 = 14; from row 2 on at least 15 younger reads, nothing to wait for)
      if (t <= 8) __builtin_amdgcn_s_waitcnt(0xC07F | (14 << 8));
      mfma16_acc(acc[i][j], fw0[j], fa0[i]);
      if (t == 0) {
        fa1[0] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + rd1);
      } else if (t < 9) {
        fw1[t - 1] = *reinterpret_cast<const s16x8_t*>(cur + w_rd + (t - 1) * 2048 + rd1);
      } else if (t < 16) {
        fa1[t - 8] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (t - 8) * 2048 + rd1);
      } else if (t == 40) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of buffer b retired
        bar();
      } else if (t > 40 && (t - 41) % 3 == 0) {
        dma(kt + 2, (t - 41) / 3, false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- half 1: set 1; W pieces of step kt + 2; wait step kt + 1; reads of its set 0
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      mfma16_acc(acc[i][j], fw1[j], fa1[i]);
      if (t < 36 && t % 5 == 0) {
        dma(kt + 2, t / 5, true);
      } else if (t == RB6 - 1) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step kt+1 landed (this step's 16 in flight)
        bar();
      } else if (t == RB6) {
        fa0[0] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + rd0);
      } else if (t > RB6 && t < RB6 + 9) {
        fw0[t - RB6 - 1] = *reinterpret_cast<const s16x8_t*>(nxt + w_rd + (t - RB6 - 1) * 2048 + rd0);
      } else if (t >= RB6 + 9 && t < RB6 + 16) {
        fa0[t - RB6 - 8] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (t - RB6 - 8) * 2048 + rd0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  mfma_drain();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (EPI == EPI_F32) {
    float* wt = ws + ((int64_t)split * tail + t_local) * (BM * BN);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = wr * 128 + 16 * i + fr, col = wc * 128 + 16 * j + 4 * fq;
        *reinterpret_cast<f32x4_t*>(wt + row * BN + col) = acc[i][j];
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
      p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
    }
  __syncthreads();
  if constexpr (EPI == EPI_NONE) {
#pragma unroll 4
    for (int it = 0; it < 32; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int m = m0 + wr * 128 + row;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 + wc * 128 + c * 8) = v;
    }
  } else {
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
      if (m < M) *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + n0 / 2 + c * 8) = pack8(of);
    }
  }
}

// ---------------------------------------------------------------------------
// Variant 6 ("persistent PGR2"): variant 3's K-loop, but each workgroup walks a
// list of tiles (tile b, b + P, b + 2P, ... of the data-parallel range; P = min(#tiles,
// 256) workgroups) as ONE continuous stream of K-steps: the LDS-DMA of step g + 2
// and the fragment reads of step g + 1 run straight across tile boundaries, so the
// next tile's first two K-steps load while the current tile finishes - no per-tile
// prologue wait (an HBM round trip, ~2-4 % of a 128-step tile). The epilogue stores
// straight from the accumulators (no LDS: both LDS buffers hold the next tile then):
// each lane owns 4 consecutive columns of a row, 8-B stores. EPI_SILU_STD maps
// each wave to 64 gate + the matching 64 up columns (W fragments 0-3 from gate rows,
// 4-7 from up rows), so silu(g) * u is formed in registers.
template <int EPI>
__global__ __launch_bounds__(NT6, 1) void pgemm7_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                        const uint16_t* __restrict__ W, int64_t ldw,
                                                        uint16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        int ntiles) {
  constexpr int RB = 37;
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUF6];  // the ONLY LDS object
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int P = gridDim.x;
  const int b = xcd_remap(blockIdx.x, P);
  const int nt = (ntiles - b + P - 1) / P;  // tiles of this workgroup: b, b + P, ...
  const int nk = K / BK;
  const int S = nt * nk;                    // K-steps of this workgroup, all tiles

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, 0x7fffffff, 0x00020000);

  // per-lane DMA offsets of the tile being LOADED (advances two K-steps ahead of compute)
  uint32_t va[8], vw[8];
  auto set_dma_tile = [&](int r) {
    int tm, tn;
    tile_mn(b + min(r, nt - 1) * P, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 64 * w + 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      va[j] = tm * BM + row < M ? (uint32_t)(((tm * BM + row) * lda + c * 8) * 2) : 0x80000000u;
      const int wrow = EPI == EPI_SILU_STD ? (row < 128 ? 0 : N / 2 - 128) + tn * 128 + row : tn * BN + row;
      vw[j] = (uint32_t)((wrow * ldw + c * 8) * 2);
    }
  };
  // piece j of operand A or W of global K-step g, whose step within its tile is kt_of_g (the
  // offsets of that tile are set by set_dma_tile)
  auto dma = [&](int g, int kt_of_g, int j, bool wop) {
    const uint32_t so = (uint32_t)(kt_of_g * BK * 2);
    char* dst = lds + (g & 1) * BUF6 + (wop ? OPB6 : 0) + (8 * w + j) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wop ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             wop ? vw[j] : va[j], so, 0, 0);
  };

  const int fr = lane & 15, fq = lane >> 4;
  const int rd0 = fr * 128 + ((fq ^ ((fr >> 1) & 7)) * 16);
  const int rd1 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) * 16);
  const int a_rd = (wr * 128) * 128;
  // W fragment j of this wave: rows wc*128 + 16 j (EPI_NONE); gate rows wc*64 + 16 j (j < 4) and
  // up rows 128 + wc*64 + 16 (j - 4) (EPI_SILU_STD)
  auto w_off = [&](int j) {
    return OPB6 + (EPI == EPI_SILU_STD ? (j < 4 ? wc * 64 + 16 * j : 128 + wc * 64 + 16 * (j - 4))
                                       : wc * 128 + 16 * j) * 128;
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s16x8_t fa0[8], fw0[8], fa1[8], fw1[8];

  set_dma_tile(0);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, 0, j, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, 0, j, true);
  if (nk == 1) set_dma_tile(1);
  const int kt1 = nk == 1 ? 0 : 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, kt1, j, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, kt1, j, true);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  bar();
  fa0[0] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + rd0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fw0[i] = *reinterpret_cast<const s16x8_t*>(lds + w_off(i) + rd0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    fa0[i] = *reinterpret_cast<const s16x8_t*>(lds + a_rd + i * 2048 + rd0);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  for (int r = 0; r < nt; ++r) {
  for (int kt = 0; kt < nk; ++kt) {
    const int g = r * nk + kt;
    const char* cur = lds + (g & 1) * BUF6;
    const char* nxt = lds + ((g & 1) ^ 1) * BUF6;
    // the DMA of this step loads global step g + 2 = step kt2 of tile r2 (scalar bookkeeping, no
    // division); past the last step it re-loads the last one into a buffer nobody reads
    int kt2 = kt + 2;
    if (nk == 1) {
      kt2 = 0;
      set_dma_tile(r + 2);
    } else if (kt2 >= nk) {
      kt2 -= nk;
      if (kt2 == 0) set_dma_tile(r + 1);
    }
    if (g + 2 >= S) kt2 = nk - 1;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      if (t <= 8) __builtin_amdgcn_s_waitcnt(0xC07F | (14 << 8));
      mfma16_acc(acc[i][j], fw0[j], fa0[i]);
      if (t == 0) {
        fa1[0] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + rd1);
      } else if (t < 9) {
        fw1[t - 1] = *reinterpret_cast<const s16x8_t*>(cur + w_off(t - 1) + rd1);
      } else if (t < 16) {
        fa1[t - 8] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (t - 8) * 2048 + rd1);
      } else if (t == 40) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        bar();
      } else if (t > 40 && (t - 41) % 3 == 0) {
        dma(g + 2, kt2, (t - 41) / 3, false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      mfma16_acc(acc[i][j], fw1[j], fa1[i]);
      if (t < 36 && t % 5 == 0) {
        dma(g + 2, kt2, t / 5, true);
      } else if (t == RB - 1) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        bar();
      } else if (t == RB) {
        fa0[0] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + rd0);
      } else if (t > RB && t < RB + 9) {
        fw0[t - RB - 1] = *reinterpret_cast<const s16x8_t*>(nxt + w_off(t - RB - 1) + rd0);
      } else if (t >= RB + 9 && t < RB + 16) {
        fa0[t - RB - 8] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (t - RB - 8) * 2048 + rd0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
    {
      // tile r done: store it straight from the accumulators, then restart them
      int tm, tn;
      tile_mn(b + r * P, tiles_m, tiles_n, tm, tn);
      mfma_drain();
      __builtin_amdgcn_sched_barrier(0);
      const int mrow = tm * BM + wr * 128 + fr;
      if constexpr (EPI == EPI_NONE) {
        uint16_t* cb = C + (int64_t)tn * BN + wc * 128 + 4 * fq;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = mrow + 16 * i;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const f32x4_t v = acc[i][j];
            u32x2_t p;
            p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            if (m < M) *reinterpret_cast<u32x2_t*>(cb + (int64_t)m * ldc + 16 * j) = p;
          }
        }
      } else {
        uint16_t* cb = C + (int64_t)tn * 128 + wc * 64 + 4 * fq;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = mrow + 16 * i;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4_t gv = acc[i][j], uv = acc[i][j + 4];
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = gv[e] / (1.f + __expf(-gv[e])) * uv[e];
            u32x2_t p;
            p[0] = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
            p[1] = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
            if (m < M) *reinterpret_cast<u32x2_t*>(cb + (int64_t)m * ldc + 16 * j) = p;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write -> MFMA srcC
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// ws [nsplit][tail][256][256] fp32 partials -> C tiles tile0 .. tile0 + tail - 1 (bf16, rows < M)
__global__ __launch_bounds__(256) void pgemm_splitk_reduce(const float* __restrict__ ws, int nsplit, int tail,
                                                           int tile0, uint16_t* __restrict__ C, int64_t ldc, int M,
                                                           int N) {
  const int t = blockIdx.x / (BM / 8), rblk = blockIdx.x % (BM / 8);  // 8 rows per block
  int tm, tn;
  tile_mn(tile0 + t, (M + BM - 1) / BM, N / BN, tm, tn);
  const int row = rblk * 8 + (threadIdx.x >> 5), col = (threadIdx.x & 31) * 8;
  const int m = tm * BM + row;
  if (m >= M) return;
  float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int s = 0; s < nsplit; ++s) {
    const float* p = ws + ((int64_t)s * tail + t) * (BM * BN) + row * BN + col;
    const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p), b = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[e] += a[e];
      f[4 + e] += b[e];
    }
  }
  *reinterpret_cast<u32x4_t*>(C + (int64_t)m * ldc + tn * BN + col) = pack8(f);
}

constexpr int PG_CUS = 256;  // MI355X compute units: one 256 x 256 tile per CU per wave

// tail split plan of the 4-wave kernel: (tiles run data-parallel, tail tiles, splits) or splits 1
__host__ inline void pgemm_plan(int M, int N, int K, int epi, int& full, int& tail, int& nsplit) {
  const int ntiles = ((M + BM - 1) / BM) * (N / BN), nk = K / BK;
  full = ntiles;
  tail = 0;
  nsplit = 1;
  const int t = ntiles % PG_CUS;
  // a last wave at most half full, and K long enough that a quarter of it still pipelines
  if (epi != EPI_NONE || t == 0 || 2 * t > PG_CUS || nk < 32) return;
  int s = PG_CUS / t;
  s = std::min(s, nk / 8);
  if (s < 2) return;
  full = ntiles - t;
  tail = t;
  nsplit = s;
}

}  // namespace

extern "C" int64_t llmd_pgemm_ws_bytes(int M, int N, int K, int epi, int variant) {
  if (M <= 0 || N % BN || K % BK) return 0;
  int full, tail, nsplit;
  pgemm_plan(M, N, K, epi, full, tail, nsplit);
  return nsplit > 1 ? (int64_t)nsplit * tail * BM * BN * 4 : 0;
}

// variant 0: 8-wave staggered 4-phase kernel; 1: 4-wave 128 x 128-per-wave kernel (+ split-K tail when
// ws is given: see pgemm_plan)
extern "C" int llmd_pgemm(const void* A, int64_t lda, const void* W, int64_t ldw, void* C, int64_t ldc, int M, int N,
                          int K, int epi, int variant, void* ws, hipStream_t st) {
  if (M <= 0) return 0;
  if (N % BN || K % BK || lda % 8 || ldw % 8 || ldc % 8) return -1;
  if (epi == EPI_SILU_STD && (variant < 3 || variant > 6)) return -3;
  // 32-bit DMA offsets
  if ((int64_t)(M - 1) * lda + K > 0x7fffffffLL || (int64_t)(N - 1) * ldw + K > 0x7fffffffLL) return -2;
  const int ntiles = ((M + BM - 1) / BM) * (N / BN);
  if (variant == 6) {
    if (((int64_t)(M - 1) * lda + K) * 2 > 0x7fffffffLL || ((int64_t)(N - 1) * ldw + K) * 2 > 0x7fffffffLL) return -2;
    int full = ntiles, tail = 0, nsplit = 1;
    if (ws != nullptr) pgemm_plan(M, N, K, epi == EPI_SILU_STD ? EPI_SILU : epi, full, tail, nsplit);
    const auto* a = (const uint16_t*)A;
    const auto* w = (const uint16_t*)W;
    auto* c = (uint16_t*)C;
    const int P = std::min(full, PG_CUS);
    if (epi == EPI_SILU_STD)
      hipLaunchKernelGGL(pgemm7_kernel<EPI_SILU_STD>, dim3(P), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc, M, N, K, full);
    else if (epi == EPI_NONE && full > 0)
      hipLaunchKernelGGL(pgemm7_kernel<EPI_NONE>, dim3(P), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc, M, N, K, full);
    else if (epi != EPI_NONE)
      return -3;
    if (nsplit > 1) {
      hipLaunchKernelGGL((pgemm6_kernel<EPI_F32, 37, 0>), dim3(tail * nsplit), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc,
                         M, N, K, full, nsplit, (float*)ws);
      hipLaunchKernelGGL(pgemm_splitk_reduce, dim3(tail * (BM / 8)), dim3(256), 0, st, (const float*)ws, nsplit,
                         tail, full, c, ldc, M, N);
    }
    return (int)hipGetLastError();
  }
  if (variant >= 3 && variant <= 5) {
    // buffer offsets are 31-bit byte offsets
    if (((int64_t)(M - 1) * lda + K) * 2 > 0x7fffffffLL || ((int64_t)(N - 1) * ldw + K) * 2 > 0x7fffffffLL) return -2;
    int full = ntiles, tail = 0, nsplit = 1;
    if (ws != nullptr) pgemm_plan(M, N, K, epi, full, tail, nsplit);
    const auto* a = (const uint16_t*)A;
    const auto* w = (const uint16_t*)W;
    auto* c = (uint16_t*)C;
    // 3: reads of the next step from half-1 MFMA 37; 4: + sc1 LDS-DMA loads; 5: reads from MFMA 44
    auto launch = [&](auto k_silu, auto k_std, auto k_none, auto k_f32) {
      if (epi == EPI_SILU)
        hipLaunchKernelGGL(k_silu, dim3(full), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1, nullptr);
      else if (epi == EPI_SILU_STD)
        hipLaunchKernelGGL(k_std, dim3(full), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1, nullptr);
      else if (full > 0)
        hipLaunchKernelGGL(k_none, dim3(full), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1, nullptr);
      if (nsplit > 1) {
        hipLaunchKernelGGL(k_f32, dim3(tail * nsplit), dim3(NT6), 0, st, a, lda, w, ldw, c, ldc, M, N, K, full,
                           nsplit, (float*)ws);
        hipLaunchKernelGGL(pgemm_splitk_reduce, dim3(tail * (BM / 8)), dim3(256), 0, st, (const float*)ws, nsplit,
                           tail, full, c, ldc, M, N);
      }
    };
    if (variant == 3)
      launch(pgemm6_kernel<EPI_SILU, 37, 0>, pgemm6_kernel<EPI_SILU_STD, 37, 0>, pgemm6_kernel<EPI_NONE, 37, 0>,
             pgemm6_kernel<EPI_F32, 37, 0>);
    else if (variant == 4)
      launch(pgemm6_kernel<EPI_SILU, 37, 16>, pgemm6_kernel<EPI_SILU_STD, 37, 16>, pgemm6_kernel<EPI_NONE, 37, 16>,
             pgemm6_kernel<EPI_F32, 37, 16>);
    else
      launch(pgemm6_kernel<EPI_SILU, 44, 0>, pgemm6_kernel<EPI_SILU_STD, 44, 0>, pgemm6_kernel<EPI_NONE, 44, 0>,
             pgemm6_kernel<EPI_F32, 44, 0>);
    return (int)hipGetLastError();
  }
  if (variant == 2) {
    int full = ntiles, tail = 0, nsplit = 1;
    if (ws != nullptr) pgemm_plan(M, N, K, epi, full, tail, nsplit);
    const auto* a = (const uint16_t*)A;
    const auto* w = (const uint16_t*)W;
    auto* c = (uint16_t*)C;
    if (epi == EPI_SILU)
      hipLaunchKernelGGL(pgemm5_kernel<EPI_SILU>, dim3(full), dim3(NT5), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1,
                         nullptr);
    else if (full > 0)
      hipLaunchKernelGGL(pgemm5_kernel<EPI_NONE>, dim3(full), dim3(NT5), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1,
                         nullptr);
    if (nsplit > 1) {
      hipLaunchKernelGGL(pgemm5_kernel<EPI_F32>, dim3(tail * nsplit), dim3(NT5), 0, st, a, lda, w, ldw, c, ldc, M, N,
                         K, full, nsplit, (float*)ws);
      hipLaunchKernelGGL(pgemm_splitk_reduce, dim3(tail * (BM / 8)), dim3(256), 0, st, (const float*)ws, nsplit,
                         tail, full, c, ldc, M, N);
    }
    return (int)hipGetLastError();
  }
  if (variant == 1) {
    int full = ntiles, tail = 0, nsplit = 1;
    if (ws != nullptr) pgemm_plan(M, N, K, epi, full, tail, nsplit);
    const auto* a = (const uint16_t*)A;
    const auto* w = (const uint16_t*)W;
    auto* c = (uint16_t*)C;
    if (epi == EPI_SILU)
      hipLaunchKernelGGL(pgemm4_kernel<EPI_SILU>, dim3(full), dim3(NT4), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1,
                         nullptr);
    else if (full > 0)
      hipLaunchKernelGGL(pgemm4_kernel<EPI_NONE>, dim3(full), dim3(NT4), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1,
                         nullptr);
    if (nsplit > 1) {
      hipLaunchKernelGGL(pgemm4_kernel<EPI_F32>, dim3(tail * nsplit), dim3(NT4), 0, st, a, lda, w, ldw, c, ldc, M, N,
                         K, full, nsplit, (float*)ws);
      hipLaunchKernelGGL(pgemm_splitk_reduce, dim3(tail * (BM / 8)), dim3(256), 0, st, (const float*)ws, nsplit,
                         tail, full, c, ldc, M, N);
    }
    return (int)hipGetLastError();
  }
  int full = ntiles, tail = 0, nsplit = 1;
  if (ws != nullptr) pgemm_plan(M, N, K, epi, full, tail, nsplit);
  const auto* a = (const uint16_t*)A;
  const auto* w = (const uint16_t*)W;
  auto* c = (uint16_t*)C;
  if (epi == EPI_SILU)
    hipLaunchKernelGGL(pgemm_kernel<EPI_SILU>, dim3(full), dim3(NT), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1,
                       nullptr);
  else if (full > 0)
    hipLaunchKernelGGL(pgemm_kernel<EPI_NONE>, dim3(full), dim3(NT), 0, st, a, lda, w, ldw, c, ldc, M, N, K, 0, 1,
                       nullptr);
  if (nsplit > 1) {
    hipLaunchKernelGGL(pgemm_kernel<EPI_F32>, dim3(tail * nsplit), dim3(NT), 0, st, a, lda, w, ldw, c, ldc, M, N, K,
                       full, nsplit, (float*)ws);
    hipLaunchKernelGGL(pgemm_splitk_reduce, dim3(tail * (BM / 8)), dim3(256), 0, st, (const float*)ws, nsplit, tail,
                       full, c, ldc, M, N);
  }
  return (int)hipGetLastError();
}
