// Medium-M decode GEMM: Y[M, N] = X[M, K] . W[N, K]^T for M = 33..128 (a decode
// batch on a P/D decode replica: 64-128 rows per step), bf16 in,
// fp32 accumulate, bf16 out.
//
// Why not skinny_gemm.hip's structure: there every wave streams its own K range
// of W straight to VGPRs and loads X fragments itself, so X traffic is M / R of
// the W bytes per workgroup - fine for M <= 16, but at M = 128 the four waves of
// a 64-row tile pull 8x the W bytes of X through the CU's load path. hipBLASLt's
// decode picks (MT32x128 tiles, no K split) have the same problem at 2-3.5 TB/s
// on these shapes (profiles/decode_tp2_shard_70b.log).
//
// Here one workgroup owns BN = 64 WRB rows of W (16 WRB per wave, the waves
// split N) and all M rows of X for one K range of a split-K; per 64-deep k-step
// the W tile (BN x 128 B) and the X tile (16 MB x 128 B) are copied global -> LDS
// by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, every byte of W read once
// from HBM, X read once per workgroup from L2 in whole 128-B lines) into an
// S-stage ring of separate __shared__ arrays (the waitcnt pass then tells the
// stages apart and the counted vmcnt keeps S-1 stages in flight across the
// barrier); each wave reads its A fragments (W) and every B fragment (X) with
// ds_read_b128 and runs 2 WRB MB mfma_f32_16x16x32_bf16 per k-step.
// LDS images: 128-B rows, 16-B slot c of row r stored at c ^ ((r >> 1) & 7)
// (swizzle applied on the DMA source address; destination stays lane-linear):
// the 16 lanes of a ds_read_b128 pass (16 rows, one k chunk) hit 16 distinct
// slots of the 256-B bank row.
// Split-K partials: fp32 [split][M][N], summed and rounded by mgemm_reduce_kernel, or (LLMD_MGEMM_FIXUP,
// column-tile counts that are multiples of 8) in the kernel by the last split of each column tile
// to finish (an atomic counter per tile; the splits of a tile share an XCD, see the epilogue).
//
// fp8 (W8A8, e4m3fn, F8 = true): the same 128-B image rows hold 128 k per step;
// a lane's 16-B fragment feeds two mfma_f32_16x16x32_fp8_fp8 (its low and high
// 8 bytes - A and B lanes use the same k permutation, so each MFMA sums a
// consistent 32-k subset), and the epilogue applies the per-token activation
// scale and the per-channel weight scale (row-wise scales are constant over k,
// so split-K partials are scaled before the reduce).
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;  // 4 waves

__device__ __forceinline__ int msw(int r) { return (r >> 1) & 7; }

template <int MB, int WRB, int S>
struct Geo {
  static constexpr int BN = 64 * WRB;        // W rows per workgroup
  static constexpr int BM = 16 * MB;         // X rows (tokens) per workgroup
  static constexpr int WIMG = BN * 128;      // W image bytes per stage
  static constexpr int XIMG = BM * 128;      // X image bytes per stage
  static constexpr int STAGE = WIMG + XIMG;
  static constexpr int NW = BN / 32;         // W DMA instructions per wave per stage (1 KB = 8 rows each)
  static constexpr int NX = BM / 32;         // X DMA instructions per wave per stage
  static constexpr int P = NW + NX;          // DMA instructions per wave per stage
  static_assert(BM % 32 == 0, "MB must be even");
};

// ACT: gate/up GEMM with the SiLU-and-mul in the epilogue on the plain [gate; up] weight
// (N = 2F rows): a wave's 16 WRB image rows are F-rows f0 .. f0 + 8 WRB - 1 of gate
// (rb < WRB / 2) then the same F-rows of up, so acc[rb] and acc[rb + WRB / 2] pair
// lane-locally; Y [M, F]; whole-K tiles only (nsplit 1).
template <int MB, int WRB, int S, bool F8 = false, int POL = 0, bool ACT = false>
__global__ __launch_bounds__(NT, 1) void mgemm_kernel(const void* __restrict__ xv, int64_t x_stride,
                                                      const void* __restrict__ wv_, int64_t w_stride, int M,
                                                      int N, int K, int steps_per_split, uint16_t* __restrict__ y,
                                                      int64_t y_stride, float* __restrict__ part,
                                                      const float* __restrict__ xs, const float* __restrict__ wsc,
                                                      int* __restrict__ cnt) {
  using G = Geo<MB, WRB, S>;
  using E = typename std::conditional<F8, uint8_t, uint16_t>::type;
  constexpr int CE = 16 / sizeof(E);  // elements per 16-B chunk
  constexpr int KE = 8 * CE;          // k elements per step (one 128-B image row)
  const E* x = reinterpret_cast<const E*>(xv);
  const E* wt = reinterpret_cast<const E*>(wv_);
  __shared__ __attribute__((aligned(1024))) char st0[G::STAGE];
  __shared__ __attribute__((aligned(1024))) char st1[G::STAGE];
  __shared__ __attribute__((aligned(1024))) char st2[G::STAGE];
  __shared__ __attribute__((aligned(1024))) char st3[S > 3 ? G::STAGE : 16];
  const int tile = blockIdx.x, sp = blockIdx.y;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int ws = __builtin_amdgcn_readfirstlane(wv);
  const int row0 = tile * G::BN;
  const int nk = K / KE;
  const int s0 = sp * steps_per_split;
  const int nsteps = min(nk, s0 + steps_per_split) - s0;  // >= 1: the host plans no empty split
  LLMD_DCHECK(nsteps >= 1 && M >= 1 && M <= 16 * MB);

  // per-lane DMA source offsets (elements) inside a k-step: instruction j of the
  // stage fills image rows 8 j .. 8 j + 7; lane L -> row 8 j + L / 8, slot L % 8,
  // reading global chunk slot ^ msw(row). Wave ws issues j = ws + 4 i.
  uint32_t woff[G::NW], xoff[G::NX];
#pragma unroll
  for (int i = 0; i < G::NW; ++i) {
    const int r = 8 * (ws + 4 * i) + (lane >> 3);
    int gr;
    if constexpr (ACT) {
      constexpr int HB = 8 * WRB;  // half of a wave's rows
      const int q = r / (2 * HB), j = r % (2 * HB), F = N / 2;
      const int f = min(row0 / 2 + HB * q + (j < HB ? j : j - HB), F - 1);  // past F: dropped
      gr = (j < HB ? 0 : F) + f;
    } else {
      gr = min(row0 + r, N - 1);  // rows past N re-read the last row (result dropped)
    }
    woff[i] = (uint32_t)((int64_t)(ACT ? gr : gr - row0) * w_stride + CE * ((lane & 7) ^ msw(r)));
  }
#pragma unroll
  for (int i = 0; i < G::NX; ++i) {
    const int r = 8 * (ws + 4 * i) + (lane >> 3);
    xoff[i] = (uint32_t)((int64_t)min(r, M - 1) * x_stride + CE * ((lane & 7) ^ msw(r)));
  }
  const E* wbase = ACT ? wt : wt + (int64_t)row0 * w_stride;
  // each tile starts its K sweep at a rotated step so concurrent workgroups do
  // not stream the same k columns of W at once (DRAM channel spread)
  const int rot = nsteps > 0 ? (tile * 5) % nsteps : 0;

  auto issue = [&](char* stg, int t) {
    const int k0 = (s0 + (t + rot) % nsteps) * KE;
#pragma unroll
    for (int i = 0; i < G::NW; ++i)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(wbase + k0 + woff[i]),
                                       (void __attribute__((address_space(3)))*)(stg + 1024 * (ws + 4 * i)), 16, 0,
                                       POL);  // POL 2 = nt: every W byte is read once per step
#pragma unroll
    for (int i = 0; i < G::NX; ++i)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(x + k0 + xoff[i]),
                                       (void __attribute__((address_space(3)))*)(stg + G::WIMG + 1024 * (ws + 4 * i)),
                                       16, 0, 0);
  };

  // per-lane LDS read offsets: A (W) rows 16 (WRB wv + rb) + c16, B (X) rows
  // 16 mb + c16; k chunk 4 h + g for mfma h of the step
  int aofs[WRB][2], bofs[MB][2];
#pragma unroll
  for (int rb = 0; rb < WRB; ++rb) {
    const int r = 16 * (WRB * wv + rb) + c16;
#pragma unroll
    for (int h = 0; h < 2; ++h) aofs[rb][h] = r * 128 + 16 * ((4 * h + g) ^ msw(r));
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int r = 16 * mb + c16;
#pragma unroll
    for (int h = 0; h < 2; ++h) bofs[mb][h] = G::WIMG + r * 128 + 16 * ((4 * h + g) ^ msw(r));
  }

  f32x4_t acc[WRB][MB];
#pragma unroll
  for (int rb = 0; rb < WRB; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* stg) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (F8) {
        u32x4_t a[WRB], b[MB];
#pragma unroll
        for (int rb = 0; rb < WRB; ++rb) a[rb] = *reinterpret_cast<const u32x4_t*>(stg + aofs[rb][h]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) b[mb] = *reinterpret_cast<const u32x4_t*>(stg + bofs[mb][h]);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int rb = 0; rb < WRB; ++rb)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
              const long av = (long)(((uint64_t)a[rb][2 * hh + 1] << 32) | a[rb][2 * hh]);
              const long bv = (long)(((uint64_t)b[mb][2 * hh + 1] << 32) | b[mb][2 * hh]);
              acc[rb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av, bv, acc[rb][mb], 0, 0, 0);
            }
      } else {
        bf16x8_t a[WRB], b[MB];
#pragma unroll
        for (int rb = 0; rb < WRB; ++rb) a[rb] = *reinterpret_cast<const bf16x8_t*>(stg + aofs[rb][h]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) b[mb] = *reinterpret_cast<const bf16x8_t*>(stg + bofs[mb][h]);
#pragma unroll
        for (int rb = 0; rb < WRB; ++rb)
#pragma unroll
          for (int mb = 0; mb < MB; ++mb)
            acc[rb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[mb], acc[rb][mb], 0, 0, 0);
      }
    }
  };

  // ring: stage t lives in st[t % S]; before computing t every wave waits for
  // its own DMAs of t (leaving the later stages in flight), the barrier makes
  // all waves' DMAs of t visible, then stage t + S - 1 is issued into the slot
  // computed at t - 1 (every wave is past that compute: the barrier; its
  // ds_reads are retired by the lgkmcnt(0) in front of it).
  // The steady-state loop runs only whole rounds in which every step keeps
  // S - 2 stages in flight and issues one: no branch inside it, so the waitcnt
  // pass keeps the per-slot (per-array) DMA bookkeeping instead of falling
  // back to vmcnt(0) before the LDS reads. vmcnt(n): gfx9 encoding (bits [3:0]
  // and [15:14]); lgkm/exp fields left open.
#define MG_WAIT(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
#define MG_LGKM0() __builtin_amdgcn_s_waitcnt(0xC07F)
  auto full = [&](char* cur, char* nxt, int t) {
    MG_WAIT((S - 2) * G::P);
    MG_LGKM0();
    __builtin_amdgcn_s_barrier();
    issue(nxt, t + S - 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(cur);
  };
  auto tail = [&](char* cur, char* nxt, int t) {
    if (t >= nsteps) return;
    const int ahead = min(S - 2, nsteps - 1 - t);
    if (ahead >= 2) MG_WAIT(2 * G::P);
    else if (ahead == 1) MG_WAIT(G::P);
    else MG_WAIT(0);
    MG_LGKM0();
    __builtin_amdgcn_s_barrier();
    if (t + S - 1 < nsteps) issue(nxt, t + S - 1);
    compute(cur);
  };
  // prologue with the arrays named statically (a pointer select would hide the
  // DMA targets from the waitcnt pass and cost a vmcnt(0) at the loop head)
  // (unconditional: a stage index past nsteps wraps to a valid k-step and is
  // never computed; the last step's vmcnt(0) drains it before the exit)
  issue(st0, 0);
  issue(st1, 1);
  if constexpr (S == 4) issue(st2, 2);
  int t = 0;
  if constexpr (S == 3) {
    for (; t + 3 + 2 <= nsteps; t += 3) {
      full(st0, st2, t);
      full(st1, st0, t + 1);
      full(st2, st1, t + 2);
    }
    // < 5 steps left
    tail(st0, st2, t);
    tail(st1, st0, t + 1);
    tail(st2, st1, t + 2);
    tail(st0, st2, t + 3);
    tail(st1, st0, t + 4);
  } else {
    for (; t + 4 + 3 <= nsteps; t += 4) {
      full(st0, st3, t);
      full(st1, st0, t + 1);
      full(st2, st1, t + 2);
      full(st3, st2, t + 3);
    }
    // < 7 steps left
    tail(st0, st3, t);
    tail(st1, st0, t + 1);
    tail(st2, st1, t + 2);
    tail(st3, st2, t + 3);
    tail(st0, st3, t + 4);
    tail(st1, st0, t + 5);
    tail(st2, st1, t + 6);
  }
#undef MG_WAIT
#undef MG_LGKM0

  // acc[rb][mb][i] = Y^T[row0 + 16 (WRB wv + rb) + 4 g + i][16 mb + c16]
  if constexpr (ACT) {
    constexpr int HW = WRB / 2;
    const int F = N / 2;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = 16 * mb + c16;
      if (m >= M) continue;
#pragma unroll
      for (int rb = 0; rb < HW; ++rb) {
        const int f = row0 / 2 + 8 * WRB * wv + 16 * rb + 4 * g;
        if (f >= F) continue;  // F % 4 == 0 (host check)
        const f32x4_t gt = acc[rb][mb], up = acc[rb + HW][mb];
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = gt[i] / (1.f + __expf(-gt[i])) * up[i];
        const uint32_t lo = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
        *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + f) = make_uint2(lo, hi);
      }
    }
    return;
  }
  const bool whole = gridDim.y == 1;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = 16 * mb + c16;
    if (m >= M) continue;
#pragma unroll
    for (int rb = 0; rb < WRB; ++rb) {
      const int n = row0 + 16 * (WRB * wv + rb) + 4 * g;
      if (n >= N) continue;  // N % 4 == 0 (host check)
      f32x4_t v = acc[rb][mb];
      if constexpr (F8) {  // row-wise scales: per-token activation x per-channel weight
        const float sx = xs[m];
        const f32x4_t sw = *reinterpret_cast<const f32x4_t*>(wsc + n);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] *= sx * sw[i];
        acc[rb][mb] = v;
      }
      if (whole) {
        const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n) = make_uint2(lo, hi);
      } else {
        *reinterpret_cast<f32x4_t*>(part + ((int64_t)sp * M + m) * N + n) = v;
      }
    }
  }
  if (whole || cnt == nullptr) return;
  // split-K fixup in the kernel (no reduce launch): the last split of this column tile to
  // finish sums the others' partials into its registers and writes bf16 Y. Release: the
  // agent-scope fence writes this XCD's L2 back so another XCD's acquire sees the partials.
  // (the flag lives in stage 0: every wave is past its last LDS read at the first barrier; the
  // 4-stage 256-row ring fills all 160 KB)
  // The host passes counters only when the column-tile count is a multiple of 8: workgroups are
  // dealt round-robin over the 8 XCDs in linear order (sp * tiles + tile), so every split of a
  // tile runs on the same XCD and meets the others in that XCD's L2 - no agent-scope fence (an
  // L2 write-back per workgroup cost 8-10 ms per 70B decode step, profiles/decode_r5.txt). The
  // vector L1 writes through; this workgroup's stores are acknowledged (vmcnt 0, stores count on
  // CDNA4) before its arrival is counted, and the last split's loads miss its L1 (it never read
  // those lines) and hit L2.
  int* last = reinterpret_cast<int*>(st0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) *last = atomicAdd(cnt + tile, 1) == (int)gridDim.y - 1;
  __syncthreads();
  if (!*last) return;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = 16 * mb + c16;
    if (m >= M) continue;
#pragma unroll
    for (int rb = 0; rb < WRB; ++rb) {
      const int n = row0 + 16 * (WRB * wv + rb) + 4 * g;
      if (n >= N) continue;
      f32x4_t v = acc[rb][mb];
      for (int s2 = 0; s2 < (int)gridDim.y; ++s2)
        if (s2 != sp) v += *reinterpret_cast<const f32x4_t*>(part + ((int64_t)s2 * M + m) * N + n);
      const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n) = make_uint2(lo, hi);
    }
  }
  if (threadIdx.x == 0) cnt[tile] = 0;  // ready for the next launch on this slab (stream order)
}

__global__ __launch_bounds__(256) void mgemm_reduce_kernel(const float* __restrict__ part, int nsplit, int M, int N,
                                                           uint16_t* __restrict__ y, int64_t y_stride) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t total = (int64_t)M * N;
  if (i4 >= total) return;
  const int m = (int)(i4 / N), n = (int)(i4 % N);
  f32x4_t s = *reinterpret_cast<const f32x4_t*>(part + i4);
  for (int k = 1; k < nsplit; ++k) s += *reinterpret_cast<const f32x4_t*>(part + (int64_t)k * total + i4);
  const uint32_t lo = (uint32_t)f2bf(s[0]) | ((uint32_t)f2bf(s[1]) << 16);
  const uint32_t hi = (uint32_t)f2bf(s[2]) | ((uint32_t)f2bf(s[3]) << 16);
  *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n) = make_uint2(lo, hi);
}

// The o / down projection's split-K partials -> y = bf16(sum); residual += y (rounded to bf16);
// out = rmsnorm(residual) * gamma. One workgroup per row with 256 * VPT threads, one 8-column chunk
// each (thread t: chunk t), so a row's partials stream with 4x the loads in flight of a 256-thread
// row. Bit-identical to mgemm_reduce_kernel + rmsnorm.hip's fused_add_rms_norm (256 threads, thread i
// owning chunks i, i + 256, ..): the same roundings, and the sum of squares is formed the unfused way -
// the rounded values go through LDS and thread i accumulates its chunks c = 0 .. VPT-1 sequentially
// (same FMA chain), then the same wave sums; the extra waves add exact zeros to the block sum.
template <int VPT>
__global__ __launch_bounds__(256 * VPT) void mgemm_reduce_norm_kernel(const float* __restrict__ part, int nsplit,
                                                                      int M, int N, uint16_t* __restrict__ residual,
                                                                      int64_t res_stride,
                                                                      const uint16_t* __restrict__ gamma, float eps,
                                                                      uint16_t* __restrict__ out, int64_t out_stride) {
  constexpr int NTR = 256 * VPT;
  __shared__ float red[NTR / 64];
  __shared__ float vs[VPT > 1 ? NTR * 8 : 1];
  const int row = blockIdx.x;
  const int nchunk = N >> 3;
  const int64_t total = (int64_t)M * N;
  const int ci = threadIdx.x;
  uint16_t* rr = residual + (int64_t)row * res_stride;
  float v[8];
  float ss = 0.f;
  if (ci < nchunk) {
    const float* p = part + (int64_t)row * N + ci * 8;
    f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(p), s1 = *reinterpret_cast<const f32x4_t*>(p + 4);
    for (int k = 1; k < nsplit; ++k) {
      s0 += *reinterpret_cast<const f32x4_t*>(p + (int64_t)k * total);
      s1 += *reinterpret_cast<const f32x4_t*>(p + (int64_t)k * total + 4);
    }
    const float y[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    unpack8(pack8(y), v);  // the GEMM output as bf16
    float rf[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(rr + ci * 8), rf);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += rf[j];
    const u32x4_t pr = pack8(v);  // the residual rounded once; normalise the rounded value
    *reinterpret_cast<u32x4_t*>(rr + ci * 8) = pr;
    unpack8(pr, v);
  }
  if constexpr (VPT == 1) {
    if (ci < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) vs[j * NTR + ci] = v[j];  // [j][chunk]: conflict-free writes and reads
    __syncthreads();
    if (ci < 256) {
#pragma unroll
      for (int c = 0; c < VPT; ++c) {
        if (ci + 256 * c < nchunk) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float t = vs[j * NTR + ci + 256 * c];
            ss += t * t;
          }
        }
      }
    }
  }
  ss = block_sum<NTR>(ss, red);
  const float inv = rsqrtf(ss / (float)N + eps);
  if (ci < nchunk) {
    float wf[8], o[8];
    unpack8(*reinterpret_cast<const u32x4_t*>(gamma + ci * 8), wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j] * inv * wf[j];
    *reinterpret_cast<u32x4_t*>(out + (int64_t)row * out_stride + ci * 8) = pack8(o);
  }
}

typedef void (*mkern_t)(const void*, int64_t, const void*, int64_t, int, int, int, int, uint16_t*, int64_t,
                        float*, const float*, const float*, int*);

// X row blocks (16 rows) of the tile for M rows: 64 / 96 / 128 rows as before, and 192 / 256 (the
// 129-256-row decode batches: 256 in flight, SURVEY K08 "M <= 256"; only 1- and 2-row-block W
// tiles fit the LDS with the 32 KB X image of 256 rows)
__host__ inline int mgemm_mb(int M) { return M <= 64 ? 4 : M <= 96 ? 6 : M <= 128 ? 8 : M <= 192 ? 12 : 16; }

template <int MB, bool F8, int POL>
mkern_t pick_w(int wrb, int stages) {
  if constexpr (MB > 8) {  // 192 / 256 rows: W tiles of 64 or 128 rows, 3 stages (4 with 64-row tiles)
    if (wrb == 1) return stages == 3 ? mgemm_kernel<MB, 1, 3, F8, POL> : mgemm_kernel<MB, 1, 4, F8, POL>;
    if (wrb == 2 && stages == 3) return mgemm_kernel<MB, 2, 3, F8, POL>;
    return nullptr;
  } else {
    if (wrb == 1) return stages == 3 ? mgemm_kernel<MB, 1, 3, F8, POL> : mgemm_kernel<MB, 1, 4, F8, POL>;
    if (wrb == 2) return stages == 3 ? mgemm_kernel<MB, 2, 3, F8, POL> : mgemm_kernel<MB, 2, 4, F8, POL>;
    if (wrb == 4) {
      if (stages == 3) return mgemm_kernel<MB, 4, 3, F8, POL>;
      if constexpr (MB == 4) return mgemm_kernel<MB, 4, 4, F8, POL>;  // 160 KB: the only 4-stage ring of 256-row tiles that fits
    }
    return nullptr;
  }
}

// The W stream's LDS-DMA with the nt policy by default (LLMD_MGEMM_NT=0: default policy, for A/B).
// 70B decode batch 64 ctx 5000: 46.6-47.2 -> 44.1 ms/step (profiles/decode_nt_r4.txt): every W
// byte is read once per step and a layer's weights (1.7 GB) never fit the MALL
bool mgemm_nt() {
  static const bool v = [] {
    const char* e = getenv("LLMD_MGEMM_NT");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <bool F8, int POL>
mkern_t pick_m_pol(int mb, int wrb, int stages) {
  switch (mb) {
    case 4: return pick_w<4, F8, POL>(wrb, stages);
    case 6: return pick_w<6, F8, POL>(wrb, stages);
    case 8: return pick_w<8, F8, POL>(wrb, stages);
    case 12: return pick_w<12, F8, POL>(wrb, stages);
    case 16: return pick_w<16, F8, POL>(wrb, stages);
  }
  return nullptr;
}

template <bool F8>
mkern_t pick_m(int mb, int wrb, int stages) {
  return mgemm_nt() ? pick_m_pol<F8, 2>(mb, wrb, stages) : pick_m_pol<F8, 0>(mb, wrb, stages);
}

template <int MB, int POL>
mkern_t pick_act_w(int wrb, int stages) {
  if constexpr (MB > 8) {
    if (wrb == 2 && stages == 3) return mgemm_kernel<MB, 2, 3, false, POL, true>;
    return nullptr;
  } else {
    if (wrb == 2) return stages == 3 ? mgemm_kernel<MB, 2, 3, false, POL, true> : mgemm_kernel<MB, 2, 4, false, POL, true>;
    if (wrb == 4) {
      if (stages == 3) return mgemm_kernel<MB, 4, 3, false, POL, true>;
      if constexpr (MB == 4) return mgemm_kernel<MB, 4, 4, false, POL, true>;
    }
    return nullptr;
  }
}

template <int POL>
mkern_t pick_act_pol(int mb, int wrb, int stages) {
  switch (mb) {
    case 4: return pick_act_w<4, POL>(wrb, stages);
    case 6: return pick_act_w<6, POL>(wrb, stages);
    case 8: return pick_act_w<8, POL>(wrb, stages);
    case 12: return pick_act_w<12, POL>(wrb, stages);
    case 16: return pick_act_w<16, POL>(wrb, stages);
  }
  return nullptr;
}

}  // namespace

// LDS bytes of one (M, wrb, stages) configuration; 0 if not instantiated
extern "C" int llmd_mgemm_lds(int M, int wrb, int stages) {
  if (M < 1 || M > 256 || (wrb != 1 && wrb != 2 && wrb != 4) || (stages != 3 && stages != 4)) return 0;
  const int mb = mgemm_mb(M);
  if (mb > 8 && !(wrb == 1 || (wrb == 2 && stages == 3))) return 0;  // the instantiated 192 / 256-row forms
  const int lds = stages * (64 * wrb * 128 + 16 * mb * 128);
  return lds <= 160 * 1024 ? lds : 0;
}

// Y = X W^T, M <= 128, K % 64 == 0, N % 4 == 0; wrb: 64-row W tiles per workgroup
// (1, 2 or 4), nsplit K splits (part: nsplit * M * N fp32 when > 1), stages 3 or 4.
// cnt: nullptr = split-K partials summed by mgemm_reduce_kernel; else a zeroed int slab of >= N / (64 wrb)
// counters for the in-kernel fixup (left zeroed again)
extern "C" int llmd_mgemm(const void* x, int64_t x_stride, const void* w, int64_t w_stride, int M, int N, int K,
                          int wrb, int nsplit, int stages, void* y, int64_t y_stride, float* part, int* cnt,
                          hipStream_t st) {
  if (M < 1 || M > 256 || K % 64 != 0 || N % 4 != 0 || nsplit < 1 || x_stride % 8 || w_stride % 8) return -1;
  if (llmd_mgemm_lds(M, wrb, stages) == 0) return -1;
  const int mb = mgemm_mb(M);
  mkern_t k = pick_m<false>(mb, wrb, stages);
  if (k == nullptr) return -2;
  const int nk = K / 64;
  const int per = (nk + nsplit - 1) / nsplit;
  nsplit = (nk + per - 1) / per;  // no empty splits
  const int bn = 64 * wrb;
  dim3 grid((N + bn - 1) / bn, nsplit);
  if (grid.x % 8) cnt = nullptr;  // the fixup needs every split of a tile on one XCD
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, st, x, x_stride, w, w_stride, M, N, K, per, (uint16_t*)y, y_stride, part,
                     (const float*)nullptr, (const float*)nullptr, nsplit > 1 ? cnt : nullptr);
  if (nsplit > 1 && cnt == nullptr) {
    const int64_t total4 = (int64_t)M * N / 4;
    hipLaunchKernelGGL(mgemm_reduce_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, part, nsplit,
                       M, N, (uint16_t*)y, y_stride);
  }
  return (int)hipGetLastError();
}

// The split-K partials of Y = X W^T only (fp32 [nsplit][M][N] in part, no reduce): their consumer fuses
// the reduce (rope_cache.hip reduce_rope_cache_kernel for the QKV projection). Returns the split count
// after the no-empty-split clamp (>= 2), or a negative error.
extern "C" int llmd_mgemm_partials(const void* x, int64_t x_stride, const void* w, int64_t w_stride, int M, int N,
                                   int K, int wrb, int nsplit, int stages, float* part, hipStream_t st) {
  if (M < 1 || M > 128 || K % 64 != 0 || N % 8 != 0 || nsplit < 2 || x_stride % 8 || w_stride % 8) return -1;
  if (llmd_mgemm_lds(M, wrb, stages) == 0) return -1;
  const int mb = mgemm_mb(M);
  mkern_t k = pick_m<false>(mb, wrb, stages);
  if (k == nullptr) return -2;
  const int nk = K / 64;
  const int per = (nk + nsplit - 1) / nsplit;
  nsplit = (nk + per - 1) / per;
  if (nsplit < 2) return -3;
  const int bn = 64 * wrb;
  dim3 grid((N + bn - 1) / bn, nsplit);
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, st, x, x_stride, w, w_stride, M, N, K, per, (uint16_t*)nullptr,
                     (int64_t)0, part, (const float*)nullptr, (const float*)nullptr, (int*)nullptr);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? nsplit : -(int)e - 100;
}

// out = rmsnorm(residual + X W^T) * gamma, residual updated in place (the decode step's o / down
// projection with the next residual-add + RMSNorm fused into its split-K reduce); nsplit must stay > 1
// after the no-empty-split clamp (else -3: the caller runs the plain GEMM + norm).
extern "C" int llmd_mgemm_add_rmsnorm(const void* x, int64_t x_stride, const void* w, int64_t w_stride, int M, int N,
                                      int K, int wrb, int nsplit, int stages, float* part, void* residual,
                                      int64_t res_stride, const void* gamma, float eps, void* out, int64_t out_stride,
                                      hipStream_t st) {
  if (M < 1 || M > 128 || K % 64 != 0 || N % 8 != 0 || N > 8 * 1024 || nsplit < 2 || x_stride % 8 ||
      w_stride % 8 || res_stride % 8 || out_stride % 8)
    return -1;
  if (llmd_mgemm_lds(M, wrb, stages) == 0) return -1;
  const int mb = mgemm_mb(M);
  mkern_t k = pick_m<false>(mb, wrb, stages);
  if (k == nullptr) return -2;
  const int nk = K / 64;
  const int per = (nk + nsplit - 1) / nsplit;
  nsplit = (nk + per - 1) / per;
  if (nsplit < 2) return -3;
  const int bn = 64 * wrb;
  dim3 grid((N + bn - 1) / bn, nsplit);
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, st, x, x_stride, w, w_stride, M, N, K, per, (uint16_t*)out, out_stride,
                     part, (const float*)nullptr, (const float*)nullptr, (int*)nullptr);
  const int vpt = (N / 8 + 255) / 256;  // the unfused norm's chunks per thread (its launch rounds to 1, 2, 4)
#define RN(V)                                                                                                   \
  hipLaunchKernelGGL((mgemm_reduce_norm_kernel<V>), dim3(M), dim3(256 * V), 0, st, (const float*)part, nsplit, M, \
                     N, (uint16_t*)residual, res_stride, (const uint16_t*)gamma, eps, (uint16_t*)out, out_stride)
  if (vpt <= 1) RN(1);
  else if (vpt <= 2) RN(2);
  else RN(4);
#undef RN
  return (int)hipGetLastError();
}

// fp8 W8A8: Y = (Xq sx) (Wq sw)^T, e4m3fn X [M, K] with per-row scales xs [M], e4m3fn
// W [N, K] with per-channel scales ws [N]; K % 128 == 0 (128 k per 128-B image row).
extern "C" int llmd_mgemm_fp8(const void* x, int64_t x_stride, const float* xs, const void* w, int64_t w_stride,
                              const float* ws, int M, int N, int K, int wrb, int nsplit, int stages, void* y,
                              int64_t y_stride, float* part, int* cnt, hipStream_t st) {
  if (M < 1 || M > 256 || K % 128 != 0 || N % 4 != 0 || nsplit < 1 || x_stride % 16 || w_stride % 16) return -1;
  if (llmd_mgemm_lds(M, wrb, stages) == 0) return -1;
  const int mb = mgemm_mb(M);
  mkern_t k = pick_m<true>(mb, wrb, stages);
  if (k == nullptr) return -2;
  const int nk = K / 128;
  const int per = (nk + nsplit - 1) / nsplit;
  nsplit = (nk + per - 1) / per;
  const int bn = 64 * wrb;
  dim3 grid((N + bn - 1) / bn, nsplit);
  if (grid.x % 8) cnt = nullptr;
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, st, x, x_stride, w, w_stride, M, N, K, per, (uint16_t*)y, y_stride, part,
                     xs, ws, nsplit > 1 ? cnt : nullptr);
  if (nsplit > 1 && cnt == nullptr) {
    const int64_t total4 = (int64_t)M * N / 4;
    hipLaunchKernelGGL(mgemm_reduce_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, part, nsplit,
                       M, N, (uint16_t*)y, y_stride);
  }
  return (int)hipGetLastError();
}

// Y [M, F] = silu(X Wg^T) * (X Wu^T) on the plain [gate; up] weight W [N = 2F, K] (the decode
// step's gate/up projection with the activation fused: no [M, 2F] intermediate, no act launch);
// wrb 2 or 4, whole K per workgroup.
extern "C" int llmd_mgemm_silu(const void* x, int64_t x_stride, const void* w, int64_t w_stride, int M, int N,
                               int K, int wrb, int stages, void* y, int64_t y_stride, hipStream_t st) {
  if (M < 1 || M > 256 || K % 64 != 0 || N % 8 != 0 || x_stride % 8 || w_stride % 8 || y_stride % 4) return -1;
  if ((wrb != 2 && wrb != 4) || llmd_mgemm_lds(M, wrb, stages) == 0) return -1;
  if ((int64_t)N * w_stride >= 0x7fffffffLL) return -2;  // 32-bit DMA offsets from the weight base
  const int mb = mgemm_mb(M);
  mkern_t k = mgemm_nt() ? pick_act_pol<2>(mb, wrb, stages) : pick_act_pol<0>(mb, wrb, stages);
  if (k == nullptr) return -2;
  const int bn = 64 * wrb;
  dim3 grid((N + bn - 1) / bn, 1);
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, st, x, x_stride, w, w_stride, M, N, K, K / 64, (uint16_t*)y, y_stride,
                     (float*)nullptr, (const float*)nullptr, (const float*)nullptr, (int*)nullptr);
  return (int)hipGetLastError();
}
