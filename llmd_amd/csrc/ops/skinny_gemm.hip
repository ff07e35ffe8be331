// Decode GEMM: Y[M, N] = X[M, K] . W[N, K]^T for decode-sized M (1..64), bf16 in,
// fp32 accumulate, bf16 out (SURVEY K08 decode shapes: M = decode batch, N/K of
// the dense projections). At these M the op is a stream over W, so the kernel is
// built around keeping W bytes in flight with NO barrier in the main loop (a
// __syncthreads() fence waits vmcnt(0) and drains the prefetch - the reason the
// round-1 LDS-staged version streamed at 2.4-4 TB/s).
//
// Orientation Y^T = W . X^T on mfma_f32_16x16x32_bf16:
//   A = W rows, 16 B per lane straight from HBM (row r = 16 rb + lane % 16,
//       k = 8 (lane / 16) .. +7 of the current 32-wide k-step);
//   B = X rows, same 16-B fragment shape, straight from L2 (X is re-read by the
//       N / R workgroups of a K range; X/W traffic = M / R).
// Decomposition (host planner `plan`): a workgroup owns R = 16 RB output
// columns (W rows) and one K range of a split-K; its 4 waves split that range
// again in 4 and are summed through LDS at the end (a 2-level tree), so every
// wave streams whole 32-k steps of all RB row blocks. Loads run one chunk of U
// k-steps ahead in two statically indexed register sets.
// Epilogue: bf16 rows when the K range is whole (gridDim.y == 1), else fp32
// partials [split][M][N] summed and rounded by dgemm_reduce_kernel.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

template <int RB, int MB, int U, int OCC>
__global__ __launch_bounds__(NT, OCC) void dgemm_kernel(const uint16_t* __restrict__ x, int64_t x_stride,
                                                        const uint16_t* __restrict__ wt, int64_t w_stride,
                                                        int M, int N, int K, int nquad_split,
                                                        uint16_t* __restrict__ y, int64_t y_stride,
                                                        float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) f32x4_t red[2][RB][MB][64];
  const int tile = blockIdx.x, sp = blockIdx.y, nsplit = gridDim.y;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int row0 = tile * (16 * RB);
  // k range: split sp owns 256-wide blocks [q0, q1); wave wv streams its own
  // contiguous quarter of them in 64-wide steps. A step is two MFMA k-steps
  // whose two 16-B loads per lane cover both halves of one 128-B line of each
  // W row, back to back from one wave (no line shared between waves).
  const int nq = K >> 8;
  const int q0 = sp * nquad_split, q1 = min(nq, q0 + nquad_split);
  const int nqs = max(0, q1 - q0);  // 256-wide blocks in this split = 64-wide steps per wave
  const int nsteps = nqs;
  const int kbase = q0 * 256 + wv * nqs * 64 + 8 * g;

  const uint16_t* wp[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int r = min(row0 + 16 * rb + c16, N - 1);
    wp[rb] = wt + (int64_t)r * w_stride + kbase;
  }
  const uint16_t* xp[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = min(16 * mb + c16, M - 1);
    xp[mb] = x + (int64_t)m * x_stride + kbase;
  }

  f32x4_t acc[RB][MB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  u32x4_t wa[U][2][RB], xa[U][2][MB], wb[U][2][RB], xb[U][2][MB];
  // chunk = U steps starting at step s; a step past the end re-reads step 0
  // (valid memory, result unused). No branch may split the main loop: the
  // waitcnt pass then counts loads across blocks conservatively and waits for
  // the prefetched chunk as well.
  // each tile starts its sweep at a rotated step, so concurrent workgroups do
  // not all read the same k column of W (+3-19 % on the 70B shapes, a
  // power-of-two row pitch otherwise piles them onto the same DRAM channels)
  const int rot = (tile * 5) % max(1, nsteps);
  auto load = [&](int s, u32x4_t (&w_)[U][2][RB], u32x4_t (&x_)[U][2][MB]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int st = s + u < nsteps ? s + u : 0;
      st = st + rot < nsteps ? st + rot : st + rot - nsteps;
      const int64_t off = (int64_t)st * 64;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)  // (nontemporal W loads measured 10-30 % slower)
          w_[u][h][rb] = *reinterpret_cast<const u32x4_t*>(wp[rb] + off + 32 * h);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) x_[u][h][mb] = *reinterpret_cast<const u32x4_t*>(xp[mb] + off + 32 * h);
    }
  };
  auto mfma_step = [&](const u32x4_t (&w_)[2][RB], const u32x4_t (&x_)[2][MB]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, w_[h][rb]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[rb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8_t, x_[h][mb]),
                                                                acc[rb][mb], 0, 0, 0);
      }
  };
  auto compute = [&](const u32x4_t (&w_)[U][2][RB], const u32x4_t (&x_)[U][2][MB]) {
#pragma unroll
    for (int u = 0; u < U; ++u) mfma_step(w_[u], x_[u]);
  };

  // main loop: pairs of chunks, one chunk always in flight behind the one in use.
  // sched_barrier(0) pins the group order: left alone the scheduler sinks the
  // prefetch loads in between the MFMAs that need the previous chunk, and the
  // counted waits then cover the prefetch too.
  const int npair = nsteps / (2 * U);
  int s = 0;
  if (npair > 0) load(0, wa, xa);
  for (int p = 0; p < npair; ++p, s += 2 * U) {
    load(s + U, wb, xb);
    __builtin_amdgcn_sched_barrier(0);
    compute(wa, xa);
    __builtin_amdgcn_sched_barrier(0);
    load(s + 2 * U, wa, xa);  // the last pair's prefetch is clamped and wasted
    __builtin_amdgcn_sched_barrier(0);
    compute(wb, xb);
    __builtin_amdgcn_sched_barrier(0);
  }
  // tail: < 2U steps, unpipelined
  for (; s < nsteps; ++s) {
    load(s, wb, xb);
    mfma_step(wb[0], xb[0]);
  }

  // ---- sum the 4 waves: (2,3) -> LDS, (0,1) add; 1 -> LDS, 0 adds
  if (wv >= 2) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) red[wv - 2][rb][mb][lane] = acc[rb][mb];
  }
  __syncthreads();
  if (wv < 2) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc[rb][mb] += red[wv][rb][mb][lane];
  }
  __syncthreads();
  if (wv == 1) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) red[0][rb][mb][lane] = acc[rb][mb];
  }
  __syncthreads();
  if (wv != 0) return;
  // acc[rb][mb][i] = Y^T[row0 + 16 rb + 4 g + i][16 mb + c16]
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = 16 * mb + c16;
    if (m >= M) continue;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const f32x4_t v = acc[rb][mb] + red[0][rb][mb][lane];
      const int n = row0 + 16 * rb + 4 * g;
      if (n >= N) continue;  // N % 4 == 0 (host check): all 4 in or all out
      if (nsplit == 1) {
        const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n) = make_uint2(lo, hi);
      } else {
        *reinterpret_cast<f32x4_t*>(part + ((int64_t)sp * M + m) * N + n) = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void dgemm_reduce_kernel(const float* __restrict__ part, int nsplit, int M, int N,
                                                           uint16_t* __restrict__ y, int64_t y_stride) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t total = (int64_t)M * N;
  if (i4 >= total) return;
  const int m = (int)(i4 / N), n = (int)(i4 % N);  // N % 4 == 0: the 4 stay in one row
  f32x4_t s = *reinterpret_cast<const f32x4_t*>(part + i4);
  for (int k = 1; k < nsplit; ++k) s += *reinterpret_cast<const f32x4_t*>(part + (int64_t)k * total + i4);
  const uint32_t lo = (uint32_t)f2bf(s[0]) | ((uint32_t)f2bf(s[1]) << 16);
  const uint32_t hi = (uint32_t)f2bf(s[2]) | ((uint32_t)f2bf(s[3]) << 16);
  *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n) = make_uint2(lo, hi);
}

// register budget per lane: the two chunk sets (2 U steps x 2 loads x (RB + MB)
// x 4) and the row pointers live in arch VGPRs (<= 256); the accumulators
// (4 RB MB) share them at two workgroups per CU, or sit in AGPRs at one
constexpr int vregs(int rb, int mb, int u) { return 16 * u * (rb + mb) + 2 * (rb + mb) + 24; }
constexpr bool fits(int rb, int mb, int u, int occ) {
  return occ == 2 ? vregs(rb, mb, u) + 4 * rb * mb <= 256 : (vregs(rb, mb, u) <= 256 && 4 * rb * mb <= 256);
}
constexpr int pick_u(int rb, int mb, int occ) { return fits(rb, mb, 2, occ) ? 2 : (fits(rb, mb, 1, occ) ? 1 : 0); }

typedef void (*kern_t)(const uint16_t*, int64_t, const uint16_t*, int64_t, int, int, int, int, uint16_t*, int64_t,
                       float*);

template <int RB, int MB>
kern_t pick(int occ) {
  if (occ == 2) {
    constexpr int u = pick_u(RB, MB, 2);
    if constexpr (u > 0) return dgemm_kernel<RB, MB, u, 2>;
    return nullptr;
  }
  constexpr int u = pick_u(RB, MB, 1);
  if constexpr (u > 0) return dgemm_kernel<RB, MB, u, 1>;
  return nullptr;
}

template <int MB>
kern_t pick_rb(int rb, int occ) {
  switch (rb) {
    case 1: return pick<1, MB>(occ);
    case 2: return pick<2, MB>(occ);
    case 3: return pick<3, MB>(occ);
    case 4: return pick<4, MB>(occ);
    case 5: return pick<5, MB>(occ);
    case 6: return pick<6, MB>(occ);
    case 7: return pick<7, MB>(occ);
    case 8: return pick<8, MB>(occ);
  }
  return nullptr;
}

kern_t pick_all(int MB, int rb, int occ) {
  return MB == 1 ? pick_rb<1>(rb, occ) : MB == 2 ? pick_rb<2>(rb, occ) : MB == 3 ? pick_rb<3>(rb, occ)
                                                                       : pick_rb<4>(rb, occ);
}

}  // namespace

// 1 if (rb, occ) has an instantiation for this M
extern "C" int llmd_dgemm_supported(int M, int rb, int occ) {
  if (M < 1 || M > 64 || rb < 1 || rb > 8 || (occ != 1 && occ != 2)) return 0;
  const int MB = (M + 15) / 16;
  return pick_u(rb, MB, occ) > 0 ? 1 : 0;
}

// Y = X W^T with a planned decomposition: rb row blocks per workgroup, nsplit
// K splits, occ workgroups per CU. part: nsplit * M * N fp32 when nsplit > 1.
extern "C" int llmd_skinny_gemm(const void* x, int64_t x_stride, const void* w, int64_t w_stride, int M, int N,
                                int K, int rb, int nsplit, int occ, void* y, int64_t y_stride, float* part,
                                hipStream_t st) {
  if (M < 1 || M > 64 || K % 256 != 0 || N % 4 != 0 || nsplit < 1 || !llmd_dgemm_supported(M, rb, occ)) return -1;
  const int nq = K / 256;
  const int per = (nq + nsplit - 1) / nsplit;
  nsplit = (nq + per - 1) / per;  // no empty splits
  const int MB = (M + 15) / 16;
  kern_t k = pick_all(MB, rb, occ);
  if (k == nullptr) return -2;
  dim3 grid((N + 16 * rb - 1) / (16 * rb), nsplit);
  hipLaunchKernelGGL(k, grid, dim3(NT), 0, st, (const uint16_t*)x, x_stride, (const uint16_t*)w, w_stride, M, N, K,
                     per, (uint16_t*)y, y_stride, part);
  if (nsplit > 1) {
    const int64_t total4 = (int64_t)M * N / 4;
    hipLaunchKernelGGL(dgemm_reduce_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, part, nsplit,
                       M, N, (uint16_t*)y, y_stride);
  }
  return (int)hipGetLastError();
}
