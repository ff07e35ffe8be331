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
    return (u + 1.f) * g / (1.f + __expf(-alpha * g));
  }
  return g / (1.f + __expf(-g)) * u;
}

template <int MODE>
__global__ __launch_bounds__(M4_NT, 1) void moe_gemm4_bf16_kernel(
    const uint16_t* __restrict__ X, int64_t x_stride, int topk, const int* __restrict__ sorted_ids,
    const int* __restrict__ tile_expert, const uint16_t* __restrict__ W, int64_t w_expert_stride, int N, int K,
    uint16_t* __restrict__ Y, int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots,
    const uint16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * M4_BUF];  // the ONLY LDS object
  const int nt_ = blockIdx.x, mt = blockIdx.y;
  const int e = tile_expert[mt];
  if (e < 0) return;
  const int m0 = mt * M4_BM, n0 = nt_ * M4_BN;
  const int nk = K / M4_BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W + (int64_t)e * w_expert_stride), 0, 0x7fffffff, 0x00020000);
  // DMA piece j of this wave: tile rows 64 w + 8 j + (lane >> 3); LDS slot lane & 7 <- chunk (lane & 7) ^ f(row)
  uint32_t va[8], vw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 64 * w + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int sid = sorted_ids[m0 + row];
    const int tok = sid < 0 ? 0 : (a_rows_are_slots ? m0 + row : sid / topk);
    va[j] = (uint32_t)(((int64_t)tok * x_stride + c * 8) * 2);
    vw[j] = (uint32_t)(((int64_t)min(n0 + row, N - 1) * K + c * 8) * 2);
  }
  auto dma = [&](int kt, int j, bool wop) {
    const uint32_t so = (uint32_t)(min(kt, nk - 1) * M4_BK * 2);
    char* dst = lds + (kt & 1) * M4_BUF + (wop ? M4_OPB : 0) + (8 * w + j) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wop ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             wop ? vw[j] : va[j], so, 0, 0);
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int rd0 = fr * 128 + ((fq ^ ((fr >> 1) & 7)) * 16);
  const int rd1 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) * 16);
  const int a_rd = (wr * 128) * 128, w_rd = M4_OPB + (wc * 128) * 128;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  s16x8_t fa0[8], fw0[8], fa1[8], fw1[8];

#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, j, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, j, true);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, j, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, j, true);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  m4_bar();
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
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write (zero init) -> MFMA srcC
  __builtin_amdgcn_sched_barrier(0);

  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = lds + (kt & 1) * M4_BUF;
    const char* nxt = lds + ((kt & 1) ^ 1) * M4_BUF;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      if (t <= 8) __builtin_amdgcn_s_waitcnt(0xC07F | (14 << 8));
      m4_mfma(acc[i][j], fw0[j], fa0[i]);
      if (t == 0) {
        fa1[0] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + rd1);
      } else if (t < 9) {
        fw1[t - 1] = *reinterpret_cast<const s16x8_t*>(cur + w_rd + (t - 1) * 2048 + rd1);
      } else if (t < 16) {
        fa1[t - 8] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (t - 8) * 2048 + rd1);
      } else if (t == 40) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        m4_bar();
      } else if (t > 40 && (t - 41) % 3 == 0) {
        dma(kt + 2, (t - 41) / 3, false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int i = t >> 3, j = t & 7;
      m4_mfma(acc[i][j], fw1[j], fa1[i]);
      if (t < 36 && t % 5 == 0) {
        dma(kt + 2, t / 5, true);
      } else if (t == M4_RB - 1) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        m4_bar();
      } else if (t == M4_RB) {
        fa0[0] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + rd0);
      } else if (t > M4_RB && t < M4_RB + 9) {
        fw0[t - M4_RB - 1] = *reinterpret_cast<const s16x8_t*>(nxt + w_rd + (t - M4_RB - 1) * 2048 + rd0);
      } else if (t >= M4_RB + 9 && t < M4_RB + 16) {
        fa0[t - M4_RB - 8] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (t - M4_RB - 8) * 2048 + rd0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // asm MFMA results -> VALU reads
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: acc[i][j][r] = C[m][n], m = wr*128 + 16 i + (lane & 15), n = wc*128 + 16 j + 4 (lane >> 4) + r
  char* img = lds + w * 32768;
  const int ncol0 = n0 + wc * 128;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 16 * i + fr, col = 16 * j + 4 * fq;
      f32x4_t v = acc[i][j];
      if (bias != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = min(ncol0 + col + r, N - 1);
          v[r] += bf2f(bias[(int64_t)e * N + n]);
        }
      }
      if constexpr (MODE == 0) {
        u32x2_t p;
        p[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        p[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<u32x2_t*>(img + row * 256 + (((col >> 3) ^ (row & 15)) * 16) + (col & 7) * 2) = p;
      } else {
        // two (g, u) pairs -> 2 outputs at half-columns col / 2, col / 2 + 1 of a [128][64] image (128-B rows)
        const float o0 = m4_act(v[0], v[1], act, alpha, limit), o1 = m4_act(v[2], v[3], act, alpha, limit);
        const uint32_t p = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
        const int hc = col >> 1;  // 0..62, even
        *reinterpret_cast<uint32_t*>(img + row * 128 + (((hc >> 3) ^ (row & 7)) * 16) + (hc & 7) * 2) = p;
      }
    }
  __syncthreads();
  if constexpr (MODE == 0) {
#pragma unroll 4
    for (int it = 0; it < 32; ++it) {
      const int row = it * 4 + (lane >> 4), c = lane & 15;
      const int p = m0 + wr * 128 + row;
      const int n = ncol0 + c * 8;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(img + row * 256 + ((c ^ (row & 15)) * 16));
      if (sorted_ids[p] >= 0 && n < N) *reinterpret_cast<u32x4_t*>(Y + (int64_t)p * y_stride + n) = v;
    }
  } else {
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int row = it * 8 + (lane >> 3), c = lane & 7;
      const int p = m0 + wr * 128 + row;
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
                                   float limit, int a_rows_are_slots, const void* bias, int64_t x_rows,
                                   hipStream_t st) {
  if (K % M4_BK || x_stride % 8 || w_expert_stride % 8 || N % 8 || (mode == 1 && N % 16)) return -1;
  // 31-bit byte offsets of the gathered rows and of one expert's weights
  if ((x_rows * x_stride + K) * 2 > 0x7fffffffLL || ((int64_t)N * K) * 2 > 0x7fffffffLL) return -2;
  if (num_tiles == 0) return 0;
  dim3 grid((N + M4_BN - 1) / M4_BN, num_tiles);
  if (mode == 0)
    hipLaunchKernelGGL(moe_gemm4_bf16_kernel<0>, grid, dim3(M4_NT), 0, st, (const uint16_t*)X, x_stride, topk,
                       sorted_ids, tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y, y_stride, act,
                       alpha, limit, a_rows_are_slots, (const uint16_t*)bias);
  else
    hipLaunchKernelGGL(moe_gemm4_bf16_kernel<1>, grid, dim3(M4_NT), 0, st, (const uint16_t*)X, x_stride, topk,
                       sorted_ids, tile_expert, (const uint16_t*)W, w_expert_stride, N, K, (uint16_t*)Y, y_stride, act,
                       alpha, limit, a_rows_are_slots, (const uint16_t*)bias);
  return (int)hipGetLastError();
}
