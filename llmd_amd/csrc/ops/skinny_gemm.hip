// Skinny (decode) GEMM: Y[M, N] = X[M, K] . W[N, K]^T for M <= 64, bf16 in,
// fp32 accumulate, bf16 out (SURVEY K08 decode shapes: M = decode batch,
// N/K = 8k..57k). At these M the op is a stream over W; hipBLASLt reaches
// ~4.5 TB/s here (profiles/r1_llama70b_decode_kernel_stats.txt), this kernel
// is built to keep more bytes in flight.
//
// Orientation Y^T = W . X^T: W rows on the MFMA M axis (A operand straight
// from HBM, 16 B per lane), the decode rows on the N axis (B operand from a
// padded LDS image of X shared by the workgroup's 4 waves).
// Workgroup = 256 W rows (wave w: rows 64w..64w+63 = 4 MFMA row blocks) x one
// K split; K advances in 128-wide stages; the next stage's W (64 VGPRs) and X
// are loaded while the current one feeds 4 x 4 x MB mfma_16x16x32_bf16.
// Epilogue: accumulators -> LDS transpose -> coalesced [M][N] rows, bf16 when
// the K range is whole, else fp32 partials reduced by skinny_reduce_kernel.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;
constexpr int ROWS = 256;          // W rows per workgroup
constexpr int KST = 128;           // K per stage
constexpr int XROW = KST * 2 + 16; // padded LDS bytes per X row (conflict-free b128 reads)

template <int MB>
__global__ __launch_bounds__(NT, (MB >= 4 ? 1 : 2)) void skinny_gemm_kernel(const uint16_t* __restrict__ x, int64_t x_stride,
                                                            const uint16_t* __restrict__ wt, int64_t w_stride,
                                                            int M, int N, int K, int stages_per_split,
                                                            uint16_t* __restrict__ y, int64_t y_stride,
                                                            float* __restrict__ part) {
  constexpr int MP = 16 * MB;  // padded M
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tile = blockIdx.x, sp = blockIdx.y, nsplit = gridDim.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int nst = K / KST;
  const int st0 = sp * stages_per_split, st1 = min(nst, st0 + stages_per_split);
  const int row_base = tile * ROWS + 64 * w;

  f32x4_t acc[4][MB];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[rb][mb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // W row pointers of this lane (A operand rows 16rb + c16), clamped in bounds
  const uint16_t* wr[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int r = min(row_base + 16 * rb + c16, N - 1);
    wr[rb] = wt + (int64_t)r * w_stride + 8 * g;
  }
  // X staging: MP rows x 128 k per stage = MP * 16 chunks of 16 B
  constexpr int XCH = MP * (KST / 8);
  constexpr int XPT = (XCH + NT - 1) / NT;
  u32x4_t xr[XPT];
  auto load_x = [&](int st) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int row = idx / (KST / 8), ch = idx % (KST / 8);
      u32x4_t v = {0, 0, 0, 0};
      if (idx < XCH && row < M) v = *reinterpret_cast<const u32x4_t*>(x + (int64_t)row * x_stride + st * KST + ch * 8);
      xr[i] = v;
    }
  };
  auto store_x = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int idx = threadIdx.x + NT * i;
      if (idx < XCH) {
        const int row = idx / (KST / 8), ch = idx % (KST / 8);
        *reinterpret_cast<u32x4_t*>(buf + row * XROW + ch * 16) = xr[i];
      }
    }
  };
  // two register sets, used alternately by an unrolled-by-2 stage loop (no
  // runtime indexing of register arrays)
  u32x4_t wa[4][4], wb[4][4];
  auto load_w = [&](int st, u32x4_t (&dst)[4][4]) {
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        dst[rb][kk] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wr[rb] + st * KST + 32 * kk));
  };
  auto compute = [&](const u32x4_t (&src)[4][4], const char* xb) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8_t xf[MB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        xf[mb] = *reinterpret_cast<const bf16x8_t*>(xb + (16 * mb + c16) * XROW + (32 * kk + 8 * g) * 2);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const bf16x8_t af = __builtin_bit_cast(bf16x8_t, src[rb][kk]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[rb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, xf[mb], acc[rb][mb], 0, 0, 0);
      }
    }
  };

  char* xb0 = smem;
  char* xb1 = smem + MP * XROW;
  if (st0 < st1) {
    load_w(st0, wa);
    load_x(st0);
    store_x(xb0);
    for (int st = st0; st < st1; st += 2) {
      // even stage: W in wa, X in xb0; prefetch st+1 into wb / xb1
      const bool m1 = st + 1 < st1;
      if (m1) {
        load_w(st + 1, wb);
        load_x(st + 1);
      }
      __syncthreads();  // xb0 of stage st visible; xb1 readers of stage st-1 done
      compute(wa, xb0);
      if (!m1) break;
      store_x(xb1);
      const bool m2 = st + 2 < st1;
      if (m2) {
        load_w(st + 2, wa);
        load_x(st + 2);
      }
      __syncthreads();
      compute(wb, xb1);
      if (m2) store_x(xb0);
    }
  }
  __syncthreads();  // X images no longer needed: reuse LDS for the transpose
  // ---- epilogue: acc[rb][mb][i] = Y^T[row_base + 16rb + 4g + i][16mb + c16]
  float* tp = reinterpret_cast<float*>(smem) + w * (MP * 64);  // [MP][64] fp32 per wave
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
      *reinterpret_cast<f32x4_t*>(tp + (16 * mb + c16) * 64 + 16 * rb + 4 * g) = acc[rb][mb];
  __syncthreads();
  // each lane writes 4 consecutive n of one m row: 16 lanes cover a 64-wide row
  for (int e = lane; e < MP * 16; e += 64) {
    const int m = e / 16, q = e % 16;
    if (m >= M) continue;
    const int n = row_base + 4 * q;
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>(tp + m * 64 + 4 * q);
    if (nsplit == 1) {
      uint16_t* yr = y + (int64_t)m * y_stride + n;
      if (n + 3 < N) {
        const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(yr) = make_uint2(lo, hi);
      } else {
        for (int j = 0; j < 4; ++j)
          if (n + j < N) yr[j] = f2bf(v[j]);
      }
    } else {
      float* pr = part + ((int64_t)sp * M + m) * N + n;
      if (n + 3 < N) {
        *reinterpret_cast<f32x4_t*>(pr) = v;
      } else {
        for (int j = 0; j < 4; ++j)
          if (n + j < N) pr[j] = v[j];
      }
    }
  }
}

__global__ __launch_bounds__(256) void skinny_reduce_kernel(const float* __restrict__ part, int nsplit, int M, int N,
                                                            uint16_t* __restrict__ y, int64_t y_stride) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t total = (int64_t)M * N;
  if (i4 >= total) return;
  const int m = (int)(i4 / N), n = (int)(i4 % N);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (n + 3 < N && (N % 4) == 0) {
    for (int sp = 0; sp < nsplit; ++sp) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(part + (int64_t)sp * total + i4);
      s[0] += v[0]; s[1] += v[1]; s[2] += v[2]; s[3] += v[3];
    }
    uint16_t* yr = y + (int64_t)m * y_stride + n;
    const uint32_t lo = (uint32_t)f2bf(s[0]) | ((uint32_t)f2bf(s[1]) << 16);
    const uint32_t hi = (uint32_t)f2bf(s[2]) | ((uint32_t)f2bf(s[3]) << 16);
    *reinterpret_cast<uint2*>(yr) = make_uint2(lo, hi);
  } else {
    for (int j = 0; j < 4 && i4 + j < total; ++j) {
      const int64_t idx = i4 + j;
      float a = 0.f;
      for (int sp = 0; sp < nsplit; ++sp) a += part[(int64_t)sp * total + idx];
      y[(idx / N) * y_stride + idx % N] = f2bf(a);
    }
  }
}

}  // namespace

extern "C" int llmd_skinny_lds_bytes(int M) {
  const int MB = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int xb = 2 * 16 * MB * XROW, tb = 4 * 16 * MB * 64 * 4;
  return xb > tb ? xb : tb;
}

extern "C" int llmd_skinny_gemm(const void* x, int64_t x_stride, const void* w, int64_t w_stride, int M, int N,
                                int K, int nsplit, void* y, int64_t y_stride, float* part, hipStream_t st) {
  if (M < 1 || M > 64 || K % KST != 0 || nsplit < 1) return -1;
  const int nst = K / KST;
  const int per = (nst + nsplit - 1) / nsplit;
  nsplit = (nst + per - 1) / per;  // no empty splits
  const int lds = llmd_skinny_lds_bytes(M);
  dim3 grid((N + ROWS - 1) / ROWS, nsplit);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)skinny_gemm_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    attr = true;
  }
  if (M <= 16)
    hipLaunchKernelGGL(skinny_gemm_kernel<1>, grid, dim3(NT), lds, st, (const uint16_t*)x, x_stride,
                       (const uint16_t*)w, w_stride, M, N, K, per, (uint16_t*)y, y_stride, part);
  else if (M <= 32)
    hipLaunchKernelGGL(skinny_gemm_kernel<2>, grid, dim3(NT), lds, st, (const uint16_t*)x, x_stride,
                       (const uint16_t*)w, w_stride, M, N, K, per, (uint16_t*)y, y_stride, part);
  else
    hipLaunchKernelGGL(skinny_gemm_kernel<4>, grid, dim3(NT), lds, st, (const uint16_t*)x, x_stride,
                       (const uint16_t*)w, w_stride, M, N, K, per, (uint16_t*)y, y_stride, part);
  if (nsplit > 1) {
    const int64_t total4 = ((int64_t)M * N + 3) / 4;
    hipLaunchKernelGGL(skinny_reduce_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, part, nsplit,
                       M, N, (uint16_t*)y, y_stride);
  }
  return (int)hipGetLastError();
}
