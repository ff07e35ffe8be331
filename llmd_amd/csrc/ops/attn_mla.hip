// Multi-head latent attention (DeepSeek-V2/V3 MLA) over a paged
// latent cache, in the weight-absorbed form: every query row carries per-head
// 576-d queries [W_UK-absorbed q_nope (512) | roped q_pe (64)] against ONE
// shared 576-d key per token [c_kv (512) | k_pe (64)]; the value is c_kv.
// The same kernel serves decode (one row per sequence) and prefill (one row
// per query token, row_len = position + 1) - MQA with a 128-head group.
//
// v1 (H not 64/128, or LLMD_MLA_V1=1). Grid (split, head group of 16, row); 256 threads = 4 waves cooperating on a
// 64-key tile staged once in LDS (576 bf16 per key, rows padded to 1168 B so
// 16-row ds_read_b128 are conflict-free):
//   S^T[key][head] : wave w takes keys 16w..16w+15, 18 x mfma_16x16x32_bf16
//                    (A = K rows from LDS, B = Q fragments in registers)
//   softmax        : per-head max / sum exchanged through LDS (4 floats x 16
//                    heads per wave), lazy O rescale (threshold 2^8)
//   O[head][dim]   : wave w owns dims 128w..128w+127, 16 MFMAs per tile
//                    (A = P[head][key] from LDS, B = c_kv^T via ds_read_b64_tr_b16)
// The next tile is prefetched into registers while the current one computes.
// nsplit > 1 writes unnormalised partials (O, max, sum in log2 units) merged
// by mla_reduce_kernel.
#include <cstdlib>
#include <type_traits>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;
constexpr int DQK = 576, DV = 512;
constexpr int ROWB = DQK * 2 + 16;       // padded LDS row bytes
constexpr int KTILE = 64 * ROWB;         // 74,752 B
constexpr int PIMG = 16 * 64 * 2;        // P[head][key] bf16
constexpr int CPR = DQK / 8;             // 72 16-B chunks per key
constexpr int LPT = 64 * CPR / NT;       // 18 chunks per thread per tile
constexpr float NEG_INF = -__builtin_huge_valf();

__device__ __forceinline__ int rowoff(int g) { return 4 * (g >> 1) + 8 * (g & 1); }

template <bool F8>
__global__ __launch_bounds__(NT, 1) void mla_kernel(
    const uint16_t* __restrict__ q, int64_t q_row_stride, const void* __restrict__ kcv,
    int64_t block_stride, int bs, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ row_seq, const int* __restrict__ row_len, int H, float scale_log2,
    int split_size, const int* __restrict__ split_dev, int nsplit, uint16_t* __restrict__ out,
    int64_t out_row_stride, float* __restrict__ part_o, float* __restrict__ part_ml, float kv_scale) {
  // fp8 (e4m3fn) latent caches: 8-B loads widened to bf16 when written to LDS
  using CR = typename std::conditional<F8, u32x2_t, u32x4_t>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ktile = smem;
  char* pimg = smem + KTILE;
  float* red = reinterpret_cast<float*>(pimg + PIMG);  // [2][4 waves][16 heads]

  const int sp = blockIdx.x, hg = blockIdx.y, r = blockIdx.z;
  const int len = row_len[r];
  if (split_dev) split_size = *split_dev;  // hipGraph replay: keys per split sized to this step's rows
  const int k0 = sp * split_size, k1 = min(len, k0 + split_size);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int head = hg * 16 + c16;
  const int* bt = block_tables + (int64_t)row_seq[r] * bt_stride;

  float m = NEG_INF, l = 0.f;  // per head c16 (identical in every wave)
  f32x4_t o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (k0 < k1) {
    // Q fragments (B operand): lane = head c16, dims 32s + 8g .. +7
    bf16x8_t qf[18];
    const uint16_t* qr = q + (int64_t)r * q_row_stride + (int64_t)head * DQK;
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      u32x4_t v = {0, 0, 0, 0};
      if (head < H) v = *reinterpret_cast<const u32x4_t*>(qr + 32 * s + 8 * g);
      qf[s] = __builtin_bit_cast(bf16x8_t, v);
    }
    CR kr[LPT];
    const int lbs = __builtin_ctz(bs);  // power-of-two block size (checked on the host)
    auto load_tile = [&](int ts) {
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int idx = threadIdx.x + NT * i;
        const int row = idx / CPR, ch = idx % CPR;
        int key = ts + row;
        key = key < k1 ? key : k1 - 1;
        const int64_t off = (int64_t)bt[key >> lbs] * block_stride + (int64_t)(key & (bs - 1)) * DQK + ch * 8;
        if constexpr (F8) {
          kr[i] = *reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(kcv) + off);
        } else {
          kr[i] = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(kcv) + off);
        }
      }
    };
    load_tile(k0);
    for (int ts = k0; ts < k1; ts += 64) {
      __syncthreads();  // previous tile fully consumed
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int idx = threadIdx.x + NT * i;
        const int row = idx / CPR, ch = idx % CPR;
        if constexpr (F8) {
          *reinterpret_cast<u32x4_t*>(ktile + row * ROWB + ch * 16) = fp8x8_to_bf16x8(kr[i]);
        } else {
          *reinterpret_cast<u32x4_t*>(ktile + row * ROWB + ch * 16) = kr[i];
        }
      }
      __syncthreads();
      if (ts + 64 < k1) load_tile(ts + 64);
      // ---- S^T for keys 16w .. 16w+15
      f32x4_t sc = {0.f, 0.f, 0.f, 0.f};
      const char* krow = ktile + (16 * w + c16) * ROWB;
#pragma unroll
      for (int s = 0; s < 18; ++s) {
        const bf16x8_t ka = *reinterpret_cast<const bf16x8_t*>(krow + 64 * s + 16 * g);
        sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[s], sc, 0, 0, 0);
      }
      // rows of sc: keys 16w + 4g + i, column: head c16
      float mx = NEG_INF;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = ts + 16 * w + 4 * g + i;
        sc[i] = key < k1 ? sc[i] : NEG_INF;
        mx = fmaxf(mx, sc[i]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (g == 0) red[w * 16 + c16] = mx;
      __syncthreads();
      float tm = fmaxf(fmaxf(red[c16], red[16 + c16]), fmaxf(red[32 + c16], red[48 + c16]));
      tm *= scale_log2;
      const bool grow = tm > m + 8.f;
      if (__ballot(grow) != 0) {  // wave-uniform; identical decision in all waves
        const float mnew = fmaxf(m, tm);
        const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
        l *= alpha;
        m = mnew;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
          for (int n = 0; n < 8; ++n) o[n][i] *= a;
        }
      }
      const float msub = (m == NEG_INF) ? 0.f : m;
      float ps = 0.f;
      uint16_t pb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[i], scale_log2, -msub));
        ps += p;
        pb[i] = f2bf(p);
      }
      *reinterpret_cast<uint2*>(pimg + c16 * 128 + (16 * w + 4 * g) * 2) =
          make_uint2((uint32_t)pb[0] | ((uint32_t)pb[1] << 16), (uint32_t)pb[2] | ((uint32_t)pb[3] << 16));
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      if (g == 0) red[64 + w * 16 + c16] = ps;
      __syncthreads();
      l += red[64 + c16] + red[80 + c16] + red[96 + c16] + red[112 + c16];
      // ---- O[head][dim] += P[head][key] . V[key][dim], dims 128w ..
      const int qq = c16 >> 2, pp = c16 & 3;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const char* prow = pimg + c16 * 128 + (32 * t2 + rowoff(g)) * 2;
        const uint2 plo = *reinterpret_cast<const uint2*>(prow);
        const uint2 phi = *reinterpret_cast<const uint2*>(prow + 32);
        const bf16x8_t pa = __builtin_bit_cast(bf16x8_t, u32x4_t{plo.x, plo.y, phi.x, phi.y});
        const int r0 = 32 * t2 + rowoff(g) + qq;
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          const int colb = (128 * w + 16 * n + 4 * pp) * 2;
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(ktile + r0 * ROWB + colb));
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(ktile + (r0 + 16) * ROWB + colb));
          const bf16x8_t vb = __builtin_bit_cast(
              bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
          o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[n], 0, 0, 0);
        }
      }
    }
  }
  // ---- epilogue: O rows are heads 4g + i (stats in lane 4g + i), columns dims
  if (nsplit == 1) {
    const float inv = l > 0.f ? kv_scale / l : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float f = __shfl(inv, 4 * g + i, 64);
      const int hh = hg * 16 + 4 * g + i;
      if (hh < H) {
        uint16_t* orow = out + (int64_t)r * out_row_stride + (int64_t)hh * DV + 128 * w;
#pragma unroll
        for (int n = 0; n < 8; ++n) orow[16 * n + c16] = f2bf(o[n][i] * f);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hh = hg * 16 + 4 * g + i;
      if (hh < H) {
        float* po = part_o + (((int64_t)r * H + hh) * nsplit + sp) * DV + 128 * w;
#pragma unroll
        for (int n = 0; n < 8; ++n) po[16 * n + c16] = o[n][i] * kv_scale;
      }
    }
    if (w == 0 && g == 0 && head < H) {
      float* pm = part_ml + (((int64_t)r * H + head) * nsplit + sp) * 2;
      pm[0] = m;
      pm[1] = l;
    }
  }
}

// ---------------------------------------------------------------- v2: all heads per workgroup
// Grid (split, H / (16 NW), row); NW waves, wave w of head group y owns heads
// 16 (NW y + w) .. +15
// over the whole 64-key tile, so every K/V tile is fetched from HBM/L2 once per
// row (v1 re-fetched it per 16-head group), the softmax stays inside the wave
// (P lane-local in the PV A-operand layout, no LDS round trip or cross-wave
// reduction) and there is one barrier per tile.
//   tile: 64 keys x 1152 B, no padding; 16-B chunk c of row r stored at slot
//         c ^ mla_swz(r). global_load_lds_dwordx4 (LDS-DMA) fills it
//         lane-linearly (the swizzle is applied on the SOURCE side), double
//         buffered: 2 x 73,728 B.
//   mla_swz(r) = (r & 2) | ((r >> 1) & 4) makes both the S^T A-operand reads
//   (ds_read_b128, lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...)
//   and the transposed V reads (ds_read_b64_tr_b16, 32-lane groups) cover
//   every bank exactly once (searched exhaustively over 16-row patterns).
//   per wave per tile: 72 MFMAs for S^T (4 key blocks x 18 k-steps), 64 for
//   O += P V (2 key halves x 32 dim blocks); O = 128 accumulator registers.
constexpr int V2_ROWB = DQK * 2;          // 1152 B
constexpr int V2_TILE = 64 * V2_ROWB;     // 73,728 B
constexpr int V2_UNITS = 64 * CPR;        // 4608 16-B slots = 72 DMA wave-instructions

__device__ __forceinline__ int mla_swz(int r) { return (r & 2) | ((r >> 1) & 4); }

// fp8 (e4m3fn) latent caches (F8): one bf16 tile + two 36,864-B fp8 staging
// buffers (same 147,456 B of LDS). The DMA fills the next staging buffer
// lane-linearly (unswizzled) while all threads widen the current one into the
// swizzled bf16 tile; K/V dequant (x kv_scale) is folded into the softmax
// scale and the output normalisation.
constexpr int V2_STAGE = 64 * DQK;        // fp8 tile bytes

// LDS-DMA from inline asm (llmd_common.h glds16): hipcc keeps counted lgkmcnt waits.
__device__ __forceinline__ void mla_glds16(const void* gsrc, unsigned lds_dst) { glds16(gsrc, lds_dst); }

template <int NW, bool BIG, bool F8>
__global__ __launch_bounds__(64 * NW, 1) void mla_v2_kernel(
    const uint16_t* __restrict__ q, int64_t q_row_stride, const void* __restrict__ kcv,
    int64_t block_stride, int bs, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ row_seq, const int* __restrict__ row_len, int H, float scale_log2,
    int split_size, const int* __restrict__ split_dev, int nsplit, uint16_t* __restrict__ out,
    int64_t out_row_stride, float* __restrict__ part_o, float* __restrict__ part_ml, float kv_scale) {
  __shared__ __attribute__((aligned(1024))) char buf0[V2_TILE];
  __shared__ __attribute__((aligned(1024))) char buf1[V2_TILE];
  const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
  // Two head groups (NW = 4 at H = 128) read the same K/V tiles. Workgroups are
  // handed to the 8 XCDs round-robin in id order, so the natural ids (x = split
  // fastest) put the two groups of one (split, row) on different XCDs and every
  // tile crosses HBM twice. Re-pair them: ids L and L + 8 (same XCD, one dispatch
  // round apart) are the two groups of one (split, row), so the second group's
  // tiles come out of that XCD's L2 (speed only: any placement stays correct).
  int sp = blockIdx.x, hgrp = blockIdx.y, r = blockIdx.z;
  if (gridDim.y == 2) {
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + 2 * blockIdx.z);
    const int total = gridDim.x * 2 * gridDim.z, full = total / 16 * 16;
    int pidx;
    if (L < full) {
      hgrp = (L & 15) >> 3;
      pidx = (L >> 4) * 8 + (L & 7);
    } else {
      hgrp = (L - full) & 1;
      pidx = full / 2 + ((L - full) >> 1);
    }
    sp = pidx % gridDim.x;
    r = pidx / gridDim.x;
  }
  const int len = row_len[r];
  if (split_dev) split_size = *split_dev;  // hipGraph replay: keys per split sized to this step's rows
  const int k0 = sp * split_size, k1 = min(len, k0 + split_size);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, g = lane >> 4,
            c16 = lane & 15;
  const int h0 = 16 * (NW * hgrp + w);  // this wave's first head
  const int head = h0 + c16;
  const int* bt = block_tables + (int64_t)row_seq[r] * bt_stride;
  const int lbs = __builtin_ctz(bs);

  float m = NEG_INF, l = 0.f;  // stats of head c16 of this wave
  f32x4_t o[32];
#pragma unroll
  for (int n = 0; n < 32; ++n) o[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (k0 < k1) {
    bf16x8_t qf[18];
    {
      const uint16_t* qr = q + (int64_t)r * q_row_stride + (int64_t)head * DQK;
#pragma unroll
      for (int s = 0; s < 18; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qr + 32 * s + 8 * g);
    }
    // DMA: slot u = 64 * (w + NW * k) + lane of the tile image
    auto issue = [&](char* base, int ts) {
      int64_t tile_off = 0;
      if constexpr (BIG) tile_off = (int64_t)bt[ts >> lbs] * block_stride + (int64_t)(ts & (bs - 1)) * DQK;
#pragma unroll
      for (int k = 0; k < 72 / NW; ++k) {
        const int u = 64 * (w + NW * k) + lane;
        const int row = u / CPR, ch = (u - row * CPR) ^ mla_swz(row);
        const int key = min(ts + row, k1 - 1);
        int64_t off;
        if constexpr (BIG) {
          off = tile_off + (int64_t)(key - ts) * DQK;
        } else {
          off = (int64_t)bt[key >> lbs] * block_stride + (int64_t)(key & (bs - 1)) * DQK;
        }
        mla_glds16(kc + off + ch * 8, lds_addr(base) + 1024 * (w + NW * k));
      }
    };
    // Per-lane LDS offsets. The swizzle depends on row & 15 only, so every read
    // below is one of 6 lane registers + a compile-time immediate (buffer,
    // key block, k-step, dim block), which keeps the address registers out of
    // the way of the 128 accumulators and 72 Q registers.
    //   S^T A operand: row srow (+16 b4), chunk (4s + g) ^ ssw
    //     = 4s + (g ^ (ssw & 2)) +/- (ssw & 4)   (+ for even s, - for odd s)
    //   V^T B operand: row vrow (+32 t2, +16), chunk (2n + (pp >> 1)) ^ vsw
    //     = 2 ((n & ~3) + ((n & 3) ^ (vsw >> 1))) + (pp >> 1)
    const int qq = c16 >> 2, pp = c16 & 3;
    const int srow = rowoff(c16 >> 2) + (c16 & 3), ssw = mla_swz(srow);
    const int gx = g ^ (ssw & 2);
    const int offE = srow * V2_ROWB + 16 * (gx + (ssw & 4));
    const int offO = srow * V2_ROWB + 16 * (gx - (ssw & 4));
    const int vrow = rowoff(g) + qq, vk = mla_swz(vrow) >> 1;
    int voff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) voff[j] = vrow * V2_ROWB + 8 * (pp & 1) + 16 * (pp >> 1) + 32 * (j ^ vk);
    auto compute = [&](const char* kt, int ts) {
      // ---- S^T[key][head] = K . Q^T over 576 dims
      f32x4_t sc[4];
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) {
        f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 18; ++s) {
          const char* p = kt + ((s & 1) ? offO : offE) + b4 * 16 * V2_ROWB + 64 * s;
          const bf16x8_t ka = *reinterpret_cast<const bf16x8_t*>(p);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[s], a, 0, 0, 0);
        }
        sc[b4] = a;
      }
      // rows of sc[b4]: keys ts + 16 b4 + rowoff(g) + i, column: head c16
      if (ts + 64 > k1) {
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (ts + 16 * b4 + rowoff(g) + i >= k1) sc[b4][i] = NEG_INF;
      }
      float mx = NEG_INF;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[b4][i]);
      // lane-local max decides; the cross-lane max only when a head's row grows
      // (attn_prefill.hip prefill_v2_kernel); l is a per-lane partial until the epilogue
      const float tl = mx * scale_log2;
      if (__ballot(tl > m + 8.f) != 0) {  // lazy rescale (threshold 2^8), wave-uniform
        float tm = fmaxf(tl, __shfl_xor(tl, 16, 64));
        tm = fmaxf(tm, __shfl_xor(tm, 32, 64));
        const float mnew = fmaxf(m, tm);
        const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
        l *= alpha;
        m = mnew;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
          for (int n = 0; n < 32; ++n) o[n][i] *= a;
        }
      }
      const float msub = (m == NEG_INF) ? 0.f : m;
      float ps = 0.f;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[b4][i], scale_log2, -msub));
          sc[b4][i] = p;
          ps += p;
        }
      l += ps;
      // ---- O[head][dim] += P[head][key] . V[key][dim]   (V = first 512 dims of the key row)
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        bf16x8_t pa;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[j] = (__bf16)sc[2 * t2][j];
          pa[4 + j] = (__bf16)sc[2 * t2 + 1][j];
        }
#pragma unroll
        for (int n = 0; n < 32; ++n) {
          const char* p0 = kt + voff[n & 3] + 32 * t2 * V2_ROWB + 32 * (n & ~3);
          s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
          s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * V2_ROWB));
          const bf16x8_t vb = __builtin_bit_cast(
              bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
          o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[n], 0, 0, 0);
        }
      }
    };
    const int nt = (k1 - k0 + 63) >> 6;
    if constexpr (F8) {
      const uint8_t* k8 = reinterpret_cast<const uint8_t*>(kcv);
      // 64 rows x 36 16-B units = 36 wave-instructions, unswizzled rows of 576 B
      auto issue8 = [&](char* base, int ts) {
        int64_t tile_off = 0;
        if constexpr (BIG) tile_off = (int64_t)bt[ts >> lbs] * block_stride + (int64_t)(ts & (bs - 1)) * DQK;
#pragma unroll
        for (int k = 0; k < (36 + NW - 1) / NW; ++k) {
          const int j = w + NW * k;
          if (j < 36) {
            const int u = 64 * j + lane;
            const int row = u / 36, c = u - row * 36;
            const int key = min(ts + row, k1 - 1);
            int64_t off;
            if constexpr (BIG) {
              off = tile_off + (int64_t)(key - ts) * DQK;
            } else {
              off = (int64_t)bt[key >> lbs] * block_stride + (int64_t)(key & (bs - 1)) * DQK;
            }
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(k8 + off + c * 16),
                                             (void __attribute__((address_space(3)))*)(base + 1024 * j), 16, 0, 0);
          }
        }
      };
      issue8(buf1, k0);
      for (int t = 0; t < nt; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // stage t landed; tile of t-1 fully consumed
        if (t + 1 < nt) issue8(buf1 + ((t + 1) & 1) * V2_STAGE, k0 + 64 * (t + 1));
        const char* st8 = buf1 + (t & 1) * V2_STAGE;
#pragma unroll
        for (int i = 0; i < 72 / NW; ++i) {
          const int v = threadIdx.x + 64 * NW * i;
          const int row = v / CPR, ch = v - row * CPR;
          const u32x2_t f = *reinterpret_cast<const u32x2_t*>(st8 + row * DQK + ch * 8);
          *reinterpret_cast<u32x4_t*>(buf0 + row * V2_ROWB + 16 * (ch ^ mla_swz(row))) = fp8x8_to_bf16x8(f);
        }
        __syncthreads();
        compute(buf0, k0 + 64 * t);
      }
    } else {
    issue(buf0, k0);
    for (int t = 0; t < nt; t += 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < nt) issue(buf1, k0 + 64 * (t + 1));
      compute(buf0, k0 + 64 * t);
      if (t + 1 >= nt) break;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 2 < nt) issue(buf0, k0 + 64 * (t + 2));
      compute(buf1, k0 + 64 * (t + 1));
    }
    }
  }
  // ---- epilogue: O rows are heads 16w + 4g + i (stats in lane 4g + i), columns dims 16n + c16
  l += __shfl_xor(l, 16, 64);  // the head's 4 lane partials
  l += __shfl_xor(l, 32, 64);
  if (nsplit == 1) {
    const float inv = l > 0.f ? kv_scale / l : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float f = __shfl(inv, 4 * g + i, 64);
      uint16_t* orow = out + (int64_t)r * out_row_stride + (int64_t)(h0 + 4 * g + i) * DV;
#pragma unroll
      for (int n = 0; n < 32; ++n) orow[16 * n + c16] = f2bf(o[n][i] * f);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* po = part_o + (((int64_t)r * H + h0 + 4 * g + i) * nsplit + sp) * DV;
#pragma unroll
      for (int n = 0; n < 32; ++n) po[16 * n + c16] = o[n][i] * kv_scale;
    }
    if (g == 0) {
      float* pm = part_ml + (((int64_t)r * H + head) * nsplit + sp) * 2;
      pm[0] = m;
      pm[1] = l;
    }
  }
}

// ---------------------------------------------------------------- v3: 32 heads per wave
// H = 128 in ONE workgroup of 4 waves, wave w owning heads 32w..32w+31 as two
// 16-head blocks: every K fragment (S^T A operand) and every V fragment (PV B
// operand) read from LDS feeds two MFMAs, so LDS traffic per FLOP is half of
// v2's (whose LDS-array time about equalled its MFMA time per tile) and each
// K/V tile crosses HBM once per row (v2 with 4-wave workgroups: twice).
// Registers at 1 wave/SIMD (512): O = the 256 AGPRs, owned outright by the
// generated asm of mla_v3_agpr.inc (gen_mla_v3.py: literal a[..] operands and
// clobbers; hipcc's own allocation of 256 accumulators + 144 Q registers
// re-homed and spilled hundreds of registers), Q = 144 VGPRs, scores in VGPRs
// via asm MFMAs. Fragment reads are software-pipelined 4 ahead with a
// sched_barrier per step, so the scheduler cannot hoist a tile's 200 reads.
// Same LDS tile image, DMA and fp8 staging as v2.
#include "mla_v3_agpr.inc"

// S^T accumulators in VGPRs (the 256 AGPRs hold O): a chain's first MFMA takes
// C = 0 (no zeroing VALU write ahead of it), later ones accumulate in place.
__device__ __forceinline__ void mla_mfma2_first(f32x4_t& s0, f32x4_t& s1, const bf16x8_t& k, const bf16x8_t& q0,
                                                const bf16x8_t& q1) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %2, %4, 0"
      : "=&v"(s0), "=&v"(s1)
      : "v"(k), "v"(q0), "v"(q1));
}
__device__ __forceinline__ void mla_mfma2_acc(f32x4_t& s0, f32x4_t& s1, const bf16x8_t& k, const bf16x8_t& q0,
                                              const bf16x8_t& q1) {
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %2, %4, %1"
      : "+v"(s0), "+v"(s1)
      : "v"(k), "v"(q0), "v"(q1));
}

template <bool BIG, bool F8, bool PBF = false>
__global__ __launch_bounds__(256, 1) void mla_v3_kernel(
    const uint16_t* __restrict__ q, int64_t q_row_stride, const void* __restrict__ kcv,
    int64_t block_stride, int bs, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ row_seq, const int* __restrict__ row_len, int H, float scale_log2,
    int split_size, const int* __restrict__ split_dev, int nsplit, uint16_t* __restrict__ out,
    int64_t out_row_stride, float* __restrict__ part_o, float* __restrict__ part_ml, float kv_scale) {
  constexpr int NW = 4;
  __shared__ __attribute__((aligned(1024))) char buf0[V2_TILE];
  __shared__ __attribute__((aligned(1024))) char buf1[V2_TILE];
  const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
  const int sp = blockIdx.x, r = blockIdx.z;
  const int len = row_len[r];
  if (split_dev) split_size = *split_dev;  // hipGraph replay: keys per split sized to this step's rows
  const int k0 = sp * split_size, k1 = min(len, k0 + split_size);
  // wave index as a scalar: the DMA's LDS destinations stay in SGPRs
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, g = lane >> 4,
            c16 = lane & 15;
  const int h0 = 32 * w;  // head block hb: heads h0 + 16 hb + (0..15)
  const int* bt = block_tables + (int64_t)row_seq[r] * bt_stride;
  const int lbs = __builtin_ctz(bs);

  float m[2] = {NEG_INF, NEG_INF}, l[2] = {0.f, 0.f};  // stats of head h0 + 16 hb + c16
  MLA3_ZERO_ACC();  // O = a[0:255]

  if (k0 < k1) {
    bf16x8_t qf[2][18];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const uint16_t* qr = q + (int64_t)r * q_row_stride + (int64_t)(h0 + 16 * hb + c16) * DQK;
#pragma unroll
      for (int s = 0; s < 18; ++s) qf[hb][s] = *reinterpret_cast<const bf16x8_t*>(qr + 32 * s + 8 * g);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): Q landed (see mla_v4_kernel)
    // this lane's element offset inside a 64-key tile for each of its 18 DMA pieces
    // (slot u = 64 (w + NW k) + lane of the swizzled tile image)
    // (< 36,864: two 16-bit offsets per register, 9 VGPRs)
    unsigned poff[72 / NW / 2];
#pragma unroll
    for (int k = 0; k < 72 / NW; ++k) {
      const int u = 64 * (w + NW * k) + lane;
      const int row = u / CPR, ch = (u - row * CPR) ^ mla_swz(row);
      const unsigned o = row * DQK + ch * 8;
      if (k & 1) poff[k >> 1] |= o << 16; else poff[k >> 1] = o;
    }
    auto issue = [&](char* base, int ts) {
      const unsigned l0 = lds_addr(base) + 1024 * w;
      if (BIG && ts + 64 <= k1) {  // a whole tile inside one cache block
        const uint16_t* tb = kc + (int64_t)bt[ts >> lbs] * block_stride + (int64_t)(ts & (bs - 1)) * DQK;
#pragma unroll
        for (int k = 0; k < 72 / NW; ++k)
          mla_glds16(tb + ((k & 1) ? (poff[k >> 1] >> 16) : (poff[k >> 1] & 0xffffu)), l0 + 1024 * NW * k);
        return;
      }
#pragma unroll
      for (int k = 0; k < 72 / NW; ++k) {
        int ln = lane;  // opaque: this (last-tile) path's addressing is recomputed, not hoisted and spilled
        asm volatile("" : "+v"(ln));
        const int u = 64 * (w + NW * k) + ln;
        const int row = u / CPR, ch = (u - row * CPR) ^ mla_swz(row);
        const int key = min(ts + row, k1 - 1);
        const int64_t off = (int64_t)bt[key >> lbs] * block_stride + (int64_t)(key & (bs - 1)) * DQK;
        mla_glds16(kc + off + ch * 8, l0 + 1024 * NW * k);
      }
    };
    // per-lane LDS offsets: as v2
    const int qq = c16 >> 2, pp = c16 & 3;
    const int srow = rowoff(c16 >> 2) + (c16 & 3), ssw = mla_swz(srow);
    const int gx = g ^ (ssw & 2);
    const int offE = srow * V2_ROWB + 16 * (gx + (ssw & 4));
    const int offO = srow * V2_ROWB + 16 * (gx - (ssw & 4));
    const int vrow = rowoff(g) + qq, vk = mla_swz(vrow) >> 1;
    int voff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) voff[j] = vrow * V2_ROWB + 8 * (pp & 1) + 16 * (pp >> 1) + 32 * (j ^ vk);
    auto compute = [&](const char* kt, int ts) {
      // K fragment j = 18 b4 + s (keys 16 b4.., k-step s); V fragment j = 32 t2 + n
      auto kread = [&](int j) -> bf16x8_t {
        const int b4 = j / 18, s = j % 18;
        return *reinterpret_cast<const bf16x8_t*>(kt + ((s & 1) ? offO : offE) + b4 * 16 * V2_ROWB + 64 * s);
      };
      auto vread = [&](int j) -> bf16x8_t {
        const int t2 = j >> 5, n = j & 31;
        const char* p0 = kt + voff[n & 3] + 32 * t2 * V2_ROWB + 32 * (n & ~3);
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * V2_ROWB));
        return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      };
      // ---- S^T[key][head] = K . Q^T over 576 dims, two head blocks per K fragment
      f32x4_t sc[2][4];
      bf16x8_t kr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) kr[j] = kread(j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) {
#pragma unroll
        for (int s = 0; s < 18; ++s) {
          const int j = 18 * b4 + s;
          const bf16x8_t ka = kr[j & 3];
          if (j + 4 < 72) kr[j & 3] = kread(j + 4);
          if (s == 0)
            mla_mfma2_first(sc[0][b4], sc[1][b4], ka, qf[0][s], qf[1][s]);
          else
            mla_mfma2_acc(sc[0][b4], sc[1][b4], ka, qf[0][s], qf[1][s]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // score MFMAs (asm) -> softmax VALU reads
      // rows of sc[hb][b4]: keys ts + 16 b4 + rowoff(g) + i, column: head h0 + 16 hb + c16
      if (ts + 64 > k1) {
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (ts + 16 * b4 + rowoff(g) + i >= k1) sc[hb][b4][i] = NEG_INF;
      }
      bf16x8_t pa[2][2];
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float mx = NEG_INF;
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[hb][b4][i]);
        const float tl = mx * scale_log2;
        if (__ballot(tl > m[hb] + 8.f) != 0) {  // lazy rescale (threshold 2^8), wave-uniform
          float tm = fmaxf(tl, __shfl_xor(tl, 16, 64));
          tm = fmaxf(tm, __shfl_xor(tm, 32, 64));
          const float mnew = fmaxf(m[hb], tm);
          const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m[hb] - mnew);
          l[hb] *= alpha;
          m[hb] = mnew;
          const float a0 = __shfl(alpha, 4 * g, 64), a1 = __shfl(alpha, 4 * g + 1, 64),
                      a2 = __shfl(alpha, 4 * g + 2, 64), a3 = __shfl(alpha, 4 * g + 3, 64);
          if (hb == 0) {
            MLA3_RESCALE0(a0, a1, a2, a3);
          } else {
            MLA3_RESCALE1(a0, a1, a2, a3);
          }
        }
        const float msub = (m[hb] == NEG_INF) ? 0.f : m[hb];
        float ps = 0.f;
#pragma unroll
        for (int b4 = 0; b4 < 4; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sc[hb][b4][i], scale_log2, -msub));
            sc[hb][b4][i] = p;
            ps += p;
          }
        l[hb] += ps;
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pa[hb][t2][j] = (__bf16)sc[hb][2 * t2][j];
            pa[hb][t2][4 + j] = (__bf16)sc[hb][2 * t2 + 1][j];
          }
      }
      bf16x8_t vr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) vr[j] = vread(j);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 1" ::: "memory");  // pa (VALU) -> asm MFMA operand
      __builtin_amdgcn_sched_barrier(0);
      // ---- O[head][dim] += P[head][key] . V[key][dim]   (V = first 512 dims of the key row)
      MLA3_PV_BLOCK
    };
    const int nt = (k1 - k0 + 63) >> 6;
    if constexpr (F8) {
      const uint8_t* k8 = reinterpret_cast<const uint8_t*>(kcv);
      // this lane's byte offset inside a 64-key fp8 tile for each of its 9 DMA pieces (rows of 576 B)
      int p8[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int u = 64 * (w + NW * k) + lane;
        const int row = u / 36, c = u - row * 36;
        p8[k] = row * DQK + c * 16;
      }
      auto issue8 = [&](char* base, int ts) {
        const unsigned l0 = lds_addr(base) + 1024 * w;
        if (BIG && ts + 64 <= k1) {
          const uint8_t* tb = k8 + (int64_t)bt[ts >> lbs] * block_stride + (int64_t)(ts & (bs - 1)) * DQK;
#pragma unroll
          for (int k = 0; k < 9; ++k) mla_glds16(tb + p8[k], l0 + 1024 * NW * k);
          return;
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          int ln = lane;  // opaque: the last tile's addressing is recomputed, not hoisted
          asm volatile("" : "+v"(ln));
          const int u = 64 * (w + NW * k) + ln;
          const int row = u / 36, c = u - row * 36;
          const int key = min(ts + row, k1 - 1);
          const int64_t off = (int64_t)bt[key >> lbs] * block_stride + (int64_t)(key & (bs - 1)) * DQK;
          mla_glds16(k8 + off + c * 16, l0 + 1024 * NW * k);
        }
      };
      issue8(buf1, k0);
      for (int t = 0; t < nt; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // stage t landed; tile of t-1 fully consumed
        if (t + 1 < nt) issue8(buf1 + ((t + 1) & 1) * V2_STAGE, k0 + 64 * (t + 1));
        const char* st8 = buf1 + (t & 1) * V2_STAGE;
        int tid = threadIdx.x;  // opaque: the widening addresses are recomputed per tile (no hoisted set)
        asm volatile("" : "+v"(tid));
#pragma unroll
        for (int i = 0; i < 72 / NW; ++i) {
          const int v = tid + 64 * NW * i;
          const int row = v / CPR, ch = v - row * CPR;
          const u32x2_t f = *reinterpret_cast<const u32x2_t*>(st8 + row * DQK + ch * 8);
          *reinterpret_cast<u32x4_t*>(buf0 + row * V2_ROWB + 16 * (ch ^ mla_swz(row))) = fp8x8_to_bf16x8(f);
        }
        __syncthreads();
        compute(buf0, k0 + 64 * t);
      }
    } else {
      issue(buf0, k0);
      for (int t = 0; t < nt; t += 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t + 1 < nt) issue(buf1, k0 + 64 * (t + 1));
        compute(buf0, k0 + 64 * t);
        if (t + 1 >= nt) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t + 2 < nt) issue(buf0, k0 + 64 * (t + 2));
        compute(buf1, k0 + 64 * (t + 1));
      }
    }
  }
  MLA3_DRAIN();  // last MFMAs -> accumulator reads
  // ---- epilogue: O rows are heads h0 + 16 hb + 4g + i (stats in lane 4g + i), columns dims 16n + c16
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    const int hh = h0 + 16 * hb;
    float lt = l[hb] + __shfl_xor(l[hb], 16, 64);  // the head's 4 lane partials
    lt += __shfl_xor(lt, 32, 64);
    const float inv = lt > 0.f ? kv_scale / lt : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x[32];
      if (hb == 0) {
        if (i == 0) { MLA3_READ_0_0(x) } else if (i == 1) { MLA3_READ_0_1(x) }
        else if (i == 2) { MLA3_READ_0_2(x) } else { MLA3_READ_0_3(x) }
      } else {
        if (i == 0) { MLA3_READ_1_0(x) } else if (i == 1) { MLA3_READ_1_1(x) }
        else if (i == 2) { MLA3_READ_1_2(x) } else { MLA3_READ_1_3(x) }
      }
      if (nsplit == 1) {
        const float f = __shfl(inv, 4 * g + i, 64);
        uint16_t* orow = out + (int64_t)r * out_row_stride + (int64_t)(hh + 4 * g + i) * DV;
#pragma unroll
        for (int n = 0; n < 32; ++n) orow[16 * n + c16] = f2bf(x[n] * f);
      } else if constexpr (PBF) {  // bf16 partials: half the split-K round trip through memory
        uint16_t* po = reinterpret_cast<uint16_t*>(part_o) + (((int64_t)r * H + hh + 4 * g + i) * nsplit + sp) * DV;
#pragma unroll
        for (int n = 0; n < 32; ++n) po[16 * n + c16] = f2bf(x[n] * kv_scale);
      } else {
        float* po = part_o + (((int64_t)r * H + hh + 4 * g + i) * nsplit + sp) * DV;
#pragma unroll
        for (int n = 0; n < 32; ++n) po[16 * n + c16] = x[n] * kv_scale;
      }
    }
    if (nsplit > 1 && g == 0) {
      float* pm = part_ml + (((int64_t)r * H + hh + c16) * nsplit + sp) * 2;
      pm[0] = m[hb];
      pm[1] = lt;
    }
  }
}

template <bool PBF>
__global__ __launch_bounds__(128) void mla_reduce_kernel(const float* __restrict__ part_o,
                                                         const float* __restrict__ part_ml,
                                                         const int* __restrict__ row_len, int H, int nsplit,
                                                         int split_size, const int* __restrict__ split_dev,
                                                         uint16_t* __restrict__ out, int64_t out_row_stride) {
  const int hh = blockIdx.x, r = blockIdx.y;
  const int len = row_len[r];
  if (split_dev) split_size = *split_dev;
  const int nact = min(nsplit, (len + split_size - 1) / split_size);
  const int64_t base = ((int64_t)r * H + hh) * nsplit;
  float M = NEG_INF;
  for (int s = 0; s < nact; ++s) M = fmaxf(M, part_ml[(base + s) * 2]);
  float den = 0.f;
  for (int s = 0; s < nact; ++s) {
    const float ms = part_ml[(base + s) * 2];
    if (ms != NEG_INF) den += exp2f(ms - M) * part_ml[(base + s) * 2 + 1];
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  uint16_t* orow = out + (int64_t)r * out_row_stride + (int64_t)hh * DV;
  for (int d = threadIdx.x; d < DV; d += 128) {
    float acc = 0.f;
    for (int s = 0; s < nact; ++s) {
      const float ms = part_ml[(base + s) * 2];
      if (ms != NEG_INF) {
        const float pv = PBF ? bf2f(reinterpret_cast<const uint16_t*>(part_o)[(base + s) * DV + d])
                             : part_o[(base + s) * DV + d];
        acc += exp2f(ms - M) * pv;
      }
    }
    orow[d] = f2bf(acc * inv);
  }
}

// ---------------------------------------------------------------- v4: v3 on a 4-deep ring of 32-key tiles
// v3's decode at rows=64 spends over half its time waiting for the next 72 KB
// tile (one tile in flight per CU, one workgroup per CU). v4 keeps v3's
// registers and math (4 waves x 32 heads, O in a[0:255], scores via VGPR asm
// MFMAs) but stages 32-key tiles (36,864 B) through a 4-slot ring: three tiles
// (108 KB) in flight while one is computed, counted vmcnt waits (9 LDS-DMA
// pieces per wave per tile) and a raw s_barrier per tile. bf16 latent caches.
constexpr int V4_TILE = 32 * V2_ROWB;  // 36,864 B
constexpr int V4_NS = 4;

template <bool BIG, bool PBF>
__global__ __launch_bounds__(256, 1) void mla_v4_kernel(
    const uint16_t* __restrict__ q, int64_t q_row_stride, const void* __restrict__ kcv,
    int64_t block_stride, int bs, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ row_seq, const int* __restrict__ row_len, int H, float scale_log2,
    int split_size, const int* __restrict__ split_dev, int nsplit, uint16_t* __restrict__ out,
    int64_t out_row_stride, float* __restrict__ part_o, float* __restrict__ part_ml, float kv_scale) {
  constexpr int NW = 4, NP = 9;  // DMA pieces per wave per tile (32 rows x 72 chunks / 256 lanes)
  __shared__ __attribute__((aligned(1024))) char ring[V4_NS * V4_TILE];
  const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
  const int sp = blockIdx.x, r = blockIdx.z;
  const int len = row_len[r];
  if (split_dev) split_size = *split_dev;
  const int k0 = sp * split_size, k1 = min(len, k0 + split_size);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, g = lane >> 4,
            c16 = lane & 15;
  const int h0 = 32 * w;
  const int* bt = block_tables + (int64_t)row_seq[r] * bt_stride;
  const int lbs = __builtin_ctz(bs);

  float m[2] = {NEG_INF, NEG_INF}, l[2] = {0.f, 0.f};
  MLA3_ZERO_ACC();

  if (k0 < k1) {
    bf16x8_t qf[2][18];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const uint16_t* qr = q + (int64_t)r * q_row_stride + (int64_t)(h0 + 16 * hb + c16) * DQK;
#pragma unroll
      for (int s = 0; s < 18; ++s) qf[hb][s] = *reinterpret_cast<const bf16x8_t*>(qr + 32 * s + 8 * g);
    }
    // Q landed before the first DMA: waited here with the builtin (hipcc sees it), its own
    // count-based waits for Q would otherwise also drain the asm DMAs issued after the loads
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    unsigned poff[(NP + 1) / 2];  // two 16-bit element offsets per register
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int u = 64 * (w + NW * k) + lane;
      const int row = u / CPR, ch = (u - row * CPR) ^ mla_swz(row);
      const unsigned o = row * DQK + ch * 8;
      if (k & 1) poff[k >> 1] |= o << 16; else poff[k >> 1] = o;
    }
    const unsigned ring0 = lds_addr(ring);
    auto issue = [&](int t) {  // tile t (keys k0 + 32 t ..) into slot t % 4: NP pieces per wave
      const int ts = k0 + 32 * t;
      const unsigned l0 = ring0 + (t & (V4_NS - 1)) * V4_TILE + 1024 * w;
      if (BIG && ts + 32 <= k1) {
        const uint16_t* tb = kc + (int64_t)bt[ts >> lbs] * block_stride + (int64_t)(ts & (bs - 1)) * DQK;
#pragma unroll
        for (int k = 0; k < NP; ++k)
          glds16(tb + ((k & 1) ? (poff[k >> 1] >> 16) : (poff[k >> 1] & 0xffffu)), l0 + 1024 * NW * k);
        return;
      }
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int u = 64 * (w + NW * k) + ln;
        const int row = u / CPR, ch = (u - row * CPR) ^ mla_swz(row);
        const int key = min(ts + row, k1 - 1);
        const int64_t off = (int64_t)bt[key >> lbs] * block_stride + (int64_t)(key & (bs - 1)) * DQK;
        glds16(kc + off + ch * 8, l0 + 1024 * NW * k);
      }
    };
    const int qq = c16 >> 2, pp = c16 & 3;
    const int srow = rowoff(c16 >> 2) + (c16 & 3), ssw = mla_swz(srow);
    const int gx = g ^ (ssw & 2);
    const int offE = srow * V2_ROWB + 16 * (gx + (ssw & 4));
    const int offO = srow * V2_ROWB + 16 * (gx - (ssw & 4));
    const int vrow = rowoff(g) + qq, vk = mla_swz(vrow) >> 1;
    int voff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) voff[j] = vrow * V2_ROWB + 8 * (pp & 1) + 16 * (pp >> 1) + 32 * (j ^ vk);
    auto compute = [&](const char* kt, int ts) {
      auto kread = [&](int j) -> bf16x8_t {  // j = 18 b4 + s, b4 in {0, 1}
        const int b4 = j / 18, s = j % 18;
        return *reinterpret_cast<const bf16x8_t*>(kt + ((s & 1) ? offO : offE) + b4 * 16 * V2_ROWB + 64 * s);
      };
      auto vread = [&](int j) -> bf16x8_t {  // j = n (one 32-key block)
        const int n = j & 31;
        const char* p0 = kt + voff[n & 3] + 32 * (n & ~3);
        s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p0);
        s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4_t*)(p0 + 16 * V2_ROWB));
        return __builtin_bit_cast(bf16x8_t, s16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      };
      f32x4_t sc[2][2];
      bf16x8_t kr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) kr[j] = kread(j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b4 = 0; b4 < 2; ++b4) {
#pragma unroll
        for (int s = 0; s < 18; ++s) {
          const int j = 18 * b4 + s;
          const bf16x8_t ka = kr[j & 3];
          if (j + 4 < 36) kr[j & 3] = kread(j + 4);
          if (s == 0)
            mla_mfma2_first(sc[0][b4], sc[1][b4], ka, qf[0][s], qf[1][s]);
          else
            mla_mfma2_acc(sc[0][b4], sc[1][b4], ka, qf[0][s], qf[1][s]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
      if (ts + 32 > k1) {
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
#pragma unroll
          for (int b4 = 0; b4 < 2; ++b4)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (ts + 16 * b4 + rowoff(g) + i >= k1) sc[hb][b4][i] = NEG_INF;
      }
      bf16x8_t pa[2][1];
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float mx = NEG_INF;
#pragma unroll
        for (int b4 = 0; b4 < 2; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[hb][b4][i]);
        const float tl = mx * scale_log2;
        if (__ballot(tl > m[hb] + 8.f) != 0) {
          float tm = fmaxf(tl, __shfl_xor(tl, 16, 64));
          tm = fmaxf(tm, __shfl_xor(tm, 32, 64));
          const float mnew = fmaxf(m[hb], tm);
          const float alpha = (mnew == NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m[hb] - mnew);
          l[hb] *= alpha;
          m[hb] = mnew;
          const float a0 = __shfl(alpha, 4 * g, 64), a1 = __shfl(alpha, 4 * g + 1, 64),
                      a2 = __shfl(alpha, 4 * g + 2, 64), a3 = __shfl(alpha, 4 * g + 3, 64);
          if (hb == 0) {
            MLA3_RESCALE0(a0, a1, a2, a3);
          } else {
            MLA3_RESCALE1(a0, a1, a2, a3);
          }
        }
        const float msub = (m[hb] == NEG_INF) ? 0.f : m[hb];
        float ps = 0.f;
#pragma unroll
        for (int b4 = 0; b4 < 2; ++b4)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sc[hb][b4][i], scale_log2, -msub));
            sc[hb][b4][i] = p;
            ps += p;
          }
        l[hb] += ps;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[hb][0][j] = (__bf16)sc[hb][0][j];
          pa[hb][0][4 + j] = (__bf16)sc[hb][1][j];
        }
      }
      bf16x8_t vr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) vr[j] = vread(j);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 1" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      MLA3_PV_BLOCK32
    };
    const int nt = (k1 - k0 + 31) >> 5;
#pragma unroll
    for (int t = 0; t < V4_NS - 1; ++t)
      if (t < nt) issue(t);
    for (int t = 0; t < nt; ++t) {
      // tile t landed for this wave (tiles issued after it may stay in flight), the raw
      // barrier extends that to every wave and retires the reads of slot (t + 3) % 4 (tile t - 1)
      if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      else if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + V4_NS - 1 < nt) issue(t + V4_NS - 1);
      compute(ring + (t & (V4_NS - 1)) * V4_TILE, k0 + 32 * t);
    }
  }
  MLA3_DRAIN();
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    const int hh = h0 + 16 * hb;
    float lt = l[hb] + __shfl_xor(l[hb], 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const float inv = lt > 0.f ? kv_scale / lt : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x[32];
      if (hb == 0) {
        if (i == 0) { MLA3_READ_0_0(x) } else if (i == 1) { MLA3_READ_0_1(x) }
        else if (i == 2) { MLA3_READ_0_2(x) } else { MLA3_READ_0_3(x) }
      } else {
        if (i == 0) { MLA3_READ_1_0(x) } else if (i == 1) { MLA3_READ_1_1(x) }
        else if (i == 2) { MLA3_READ_1_2(x) } else { MLA3_READ_1_3(x) }
      }
      if (nsplit == 1) {
        const float f = __shfl(inv, 4 * g + i, 64);
        uint16_t* orow = out + (int64_t)r * out_row_stride + (int64_t)(hh + 4 * g + i) * DV;
#pragma unroll
        for (int n = 0; n < 32; ++n) orow[16 * n + c16] = f2bf(x[n] * f);
      } else if constexpr (PBF) {
        uint16_t* po = reinterpret_cast<uint16_t*>(part_o) + (((int64_t)r * H + hh + 4 * g + i) * nsplit + sp) * DV;
#pragma unroll
        for (int n = 0; n < 32; ++n) po[16 * n + c16] = f2bf(x[n] * kv_scale);
      } else {
        float* po = part_o + (((int64_t)r * H + hh + 4 * g + i) * nsplit + sp) * DV;
#pragma unroll
        for (int n = 0; n < 32; ++n) po[16 * n + c16] = x[n] * kv_scale;
      }
    }
    if (nsplit > 1 && g == 0) {
      float* pm = part_ml + (((int64_t)r * H + hh + c16) * nsplit + sp) * 2;
      pm[0] = m[hb];
      pm[1] = lt;
    }
  }
}

// Split merge, one wave per (row, head): lane l owns dims 8l..8l+7 (16-B partial
// loads, bf16 or fp32), the split weights exp2(m_s - M) / sum are wave-uniform.
// 4 heads per 256-thread workgroup.
template <bool PBF>
__global__ __launch_bounds__(256) void mla_reduce2_kernel(const float* __restrict__ part_o,
                                                          const float* __restrict__ part_ml,
                                                          const int* __restrict__ row_len, int H, int nsplit,
                                                          int split_size, const int* __restrict__ split_dev,
                                                          uint16_t* __restrict__ out, int64_t out_row_stride) {
  const int hh = blockIdx.x * 4 + (threadIdx.x >> 6), r = blockIdx.y, lane = threadIdx.x & 63;
  if (hh >= H) return;
  const int len = row_len[r];
  if (split_dev) split_size = *split_dev;
  const int nact = min(nsplit, (len + split_size - 1) / split_size);
  const int64_t base = ((int64_t)r * H + hh) * nsplit;
  float M = NEG_INF;
  for (int s = 0; s < nact; ++s) M = fmaxf(M, part_ml[(base + s) * 2]);
  float den = 0.f;
  for (int s = 0; s < nact; ++s) {
    const float ms = part_ml[(base + s) * 2];
    if (ms != NEG_INF) den += exp2f(ms - M) * part_ml[(base + s) * 2 + 1];
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nact; ++s) {
    const float ms = part_ml[(base + s) * 2];
    if (ms == NEG_INF) continue;
    const float wgt = exp2f(ms - M) * inv;
    if constexpr (PBF) {
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(part_o) +
                                                           (base + s) * DV + 8 * lane);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += wgt * f[k];
    } else {
      const f32x4_t* pv = reinterpret_cast<const f32x4_t*>(part_o + (base + s) * DV + 8 * lane);
      const f32x4_t a = pv[0], b = pv[1];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[k] += wgt * a[k];
        acc[4 + k] += wgt * b[k];
      }
    }
  }
  *reinterpret_cast<u32x4_t*>(out + (int64_t)r * out_row_stride + (int64_t)hh * DV + 8 * lane) = pack8(acc);
}

}  // namespace

// Kernel shape for H = 128, as 10 * waves + head blocks per wave:
//   81: v2, 8 waves x 16 heads (2 waves/SIMD, register budget 256: the 128
//       accumulators + 72 Q registers spill a few dozen values);
//   41: v2, two 64-head workgroups of 4 waves x 16 heads (1 wave/SIMD, no
//       spills, each K/V tile fetched by both);
//   42: v3, one workgroup of 4 waves x 32 heads.
// Round 4 (profiles/mla_r4_shapes.txt, ctx 4096): 42 takes bf16 decode rows=64
// 0.150 -> 0.113 ms and prefill rows=2048 2.68 -> 1.49 ms (81: 2.83), fp8
// prefill 2.85 -> 2.41; at <= 16 rows 41 is as fast or faster (fp8 rows=8:
// 0.055 vs 0.069 ms).
// LLMD_MLA_SHAPE=41|42|81 forces one (LLMD_MLA_NW=4|8 is 41|81).
extern "C" int llmd_mla_v2_shape(int R, int fp8) {
  static const int forced = [] {
    const char* e = getenv("LLMD_MLA_SHAPE");
    if (e) return atoi(e);
    e = getenv("LLMD_MLA_NW");
    return e ? 10 * atoi(e) + 1 : 0;
  }();
  if (forced == 41 || forced == 42 || forced == 43 || forced == 81) return forced;
  return R <= 16 ? 41 : 42;
}

// v3 split partials in bf16 (default; LLMD_MLA_PARTIAL_BF16=0 keeps fp32): rows=64
// ctx 4k 0.112 -> 0.108 ms, MLA numerics tests pass (profiles/mla_r4_shapes.txt)
static bool mla_partial_bf16() {
  static const bool on = [] {
    const char* e = getenv("LLMD_MLA_PARTIAL_BF16");
    return !(e && e[0] == '0');
  }();
  return on;
}

// v2 (64-head groups per workgroup) for 64 or 128 heads; LLMD_MLA_V1=1 forces v1
extern "C" int llmd_mla_uses_v2(int H) {
  static const int force_v1 = [] {
    const char* e = getenv("LLMD_MLA_V1");
    return e && e[0] == '1';
  }();
  return !force_v1 && (H == 64 || H == 128);
}

extern "C" int llmd_mla_attention(const void* q, int64_t q_row_stride, const void* kc, int64_t block_stride,
                                  int bs, const int* block_tables, int bt_stride, const int* row_seq,
                                  const int* row_len, int R, int H, float scale, int split_size, int nsplit,
                                  void* out, int64_t out_row_stride, float* part_o, float* part_ml, int fp8,
                                  float kv_scale, const int* split_dev, hipStream_t st) {
  if (R == 0) return 0;
  if (split_size % 64 != 0 || nsplit < 1) return -1;
  const size_t lds = KTILE + PIMG + 128 * sizeof(float);
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)mla_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)mla_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  const float scale_log2 = scale * kv_scale * 1.4426950408889634f;
  bool pbf = false;  // v3 split partials in bf16 (LLMD_MLA_PARTIAL_BF16=1)
  if (llmd_mla_uses_v2(H)) {
#define V2(NW, BIG, F8)                                                                                        \
  hipLaunchKernelGGL((mla_v2_kernel<NW, BIG, F8>), dim3(nsplit, H / (16 * NW), R), dim3(64 * NW), 0, st,      \
                     (const uint16_t*)q, q_row_stride, kc, block_stride, bs, block_tables, bt_stride, row_seq, \
                     row_len, H, scale_log2, split_size, split_dev, nsplit, (uint16_t*)out, out_row_stride,       \
                     part_o, part_ml, kv_scale)
#define V2NW(NW)                                   \
  if (fp8) {                                       \
    if (big) V2(NW, true, true); else V2(NW, false, true);   \
  } else {                                         \
    if (big) V2(NW, true, false); else V2(NW, false, false); \
  }
#define V4(BIG)                                                                                                \
  do {                                                                                                         \
    if (pbf) V4P(BIG, true); else V4P(BIG, false);                                                             \
  } while (0)
#define V4P(BIG, P)                                                                                            \
  hipLaunchKernelGGL((mla_v4_kernel<BIG, P>), dim3(nsplit, 1, R), dim3(256), 0, st, (const uint16_t*)q,          \
                     q_row_stride, kc, block_stride, bs, block_tables, bt_stride, row_seq, row_len, H, scale_log2, \
                     split_size, split_dev, nsplit, (uint16_t*)out, out_row_stride, part_o, part_ml, kv_scale)
#define V3(BIG, F8)                                                                                            \
  if (pbf) V3P(BIG, F8, true); else V3P(BIG, F8, false)
#define V3P(BIG, F8, P)                                                                                        \
  hipLaunchKernelGGL((mla_v3_kernel<BIG, F8, P>), dim3(nsplit, 1, R), dim3(256), 0, st, (const uint16_t*)q,     \
                     q_row_stride, kc, block_stride, bs, block_tables, bt_stride, row_seq, row_len, H, scale_log2, \
                     split_size, split_dev, nsplit, (uint16_t*)out, out_row_stride, part_o, part_ml, kv_scale)
    const bool big = bs >= 64;
    const int shape = H == 128 ? llmd_mla_v2_shape(R, fp8) : 41;
    pbf = (shape == 42 || shape == 43) && nsplit > 1 && mla_partial_bf16();
    if (shape == 81) {
      V2NW(8)
    } else if (shape == 43 && !fp8) {
      if (big) V4(true); else V4(false);
    } else if (shape == 42 || shape == 43) {
      if (fp8) {
        if (big) V3(true, true); else V3(false, true);
      } else {
        if (big) V3(true, false); else V3(false, false);
      }
    } else {
      V2NW(4)
    }
#undef V3
#undef V3P
#undef V4
#undef V4P
#undef V2NW
#undef V2
  } else {
    dim3 grid(nsplit, (H + 15) / 16, R);
    if (fp8) {
      hipLaunchKernelGGL(mla_kernel<true>, grid, dim3(NT), lds, st, (const uint16_t*)q, q_row_stride, kc,
                         block_stride, bs, block_tables, bt_stride, row_seq, row_len, H, scale_log2, split_size,
                         split_dev, nsplit, (uint16_t*)out, out_row_stride, part_o, part_ml, kv_scale);
    } else {
      hipLaunchKernelGGL(mla_kernel<false>, grid, dim3(NT), lds, st, (const uint16_t*)q, q_row_stride, kc,
                         block_stride, bs, block_tables, bt_stride, row_seq, row_len, H, scale_log2, split_size,
                         split_dev, nsplit, (uint16_t*)out, out_row_stride, part_o, part_ml, kv_scale);
    }
  }
  if (nsplit > 1) {
    // the vectorised merge needs 16-B aligned output rows (out_row_stride % 8: the op checks it)
    hipLaunchKernelGGL(pbf ? mla_reduce2_kernel<true> : mla_reduce2_kernel<false>, dim3((H + 3) / 4, R), dim3(256),
                       0, st, part_o, part_ml, row_len, H, nsplit, split_size, split_dev, (uint16_t*)out,
                       out_row_stride);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// MLA rope + latent-cache write. One workgroup per token:
//   q_lat[t, h, 512:576] = rope(q[t, h, 128:192])   (GPT-J interleaved pairs)
//   cache[slot] = [kv_c[t] (512) | rope(k_pe[t]) (64)]
namespace {
template <bool F8>
__global__ __launch_bounds__(256) void mla_rope_cache_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, uint16_t* __restrict__ q_lat, int64_t ql_stride,
    const uint16_t* __restrict__ kv_c, int64_t kvc_stride, const uint16_t* __restrict__ k_pe,
    int64_t kpe_stride, const int64_t* __restrict__ positions, const float* __restrict__ cos_sin, int H,
    const int64_t* __restrict__ slots, void* __restrict__ cache, int64_t block_stride, int bs, float kv_inv) {
  const int t = blockIdx.x;
  const float* cs = cos_sin + positions[t] * 64;
  // q_pe: H heads x 32 pairs
  for (int i = threadIdx.x; i < H * 32; i += 256) {
    const int h = i >> 5, p = i & 31;
    const uint16_t* src = q + (int64_t)t * q_stride + h * 192 + 128 + 2 * p;
    const float x0 = bf2f(src[0]), x1 = bf2f(src[1]);
    const float c = cs[p], s = cs[32 + p];
    uint16_t* dst = q_lat + (int64_t)t * ql_stride + h * 576 + 512 + 2 * p;
    dst[0] = f2bf(x0 * c - x1 * s);
    dst[1] = f2bf(x0 * s + x1 * c);
  }
  const int64_t slot = slots[t];
  if (slot < 0) return;
  const int64_t roff = (slot / bs) * block_stride + (slot % bs) * 576;  // elements
  if constexpr (F8) {  // stored as saturate(x / kv_scale), 8 elements per thread
    uint8_t* row8 = reinterpret_cast<uint8_t*>(cache) + roff;
    const int i = threadIdx.x;
    float f[8];
    if (i < 64) {
      const u32x4_t v = reinterpret_cast<const u32x4_t*>(kv_c + (int64_t)t * kvc_stride)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[2 * j] = __uint_as_float(v[j] << 16) * kv_inv;
        f[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u) * kv_inv;
      }
      *reinterpret_cast<u32x2_t*>(row8 + 8 * i) = f32x8_to_fp8(f);
    } else if (i < 72) {
      const int p0 = 4 * (i - 64);  // pairs p0 .. p0+3
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = p0 + j;
        const uint16_t* src = k_pe + (int64_t)t * kpe_stride + 2 * p;
        const float x0 = bf2f(src[0]), x1 = bf2f(src[1]);
        const float c = cs[p], s = cs[32 + p];
        f[2 * j] = (x0 * c - x1 * s) * kv_inv;
        f[2 * j + 1] = (x0 * s + x1 * c) * kv_inv;
      }
      *reinterpret_cast<u32x2_t*>(row8 + 512 + 2 * p0) = f32x8_to_fp8(f);
    }
    return;
  }
  uint16_t* row = reinterpret_cast<uint16_t*>(cache) + roff;
  for (int i = threadIdx.x; i < 512 / 8; i += 256)
    reinterpret_cast<u32x4_t*>(row)[i] = reinterpret_cast<const u32x4_t*>(kv_c + (int64_t)t * kvc_stride)[i];
  if (threadIdx.x < 32) {
    const int p = threadIdx.x;
    const uint16_t* src = k_pe + (int64_t)t * kpe_stride + 2 * p;
    const float x0 = bf2f(src[0]), x1 = bf2f(src[1]);
    const float c = cs[p], s = cs[32 + p];
    row[512 + 2 * p] = f2bf(x0 * c - x1 * s);
    row[512 + 2 * p + 1] = f2bf(x0 * s + x1 * c);
  }
}
}  // namespace

extern "C" int llmd_mla_rope_cache(const void* q, int64_t q_stride, void* q_lat, int64_t ql_stride, const void* kv_c,
                                   int64_t kvc_stride, const void* k_pe, int64_t kpe_stride, const int64_t* positions,
                                   const float* cos_sin, int T, int H, const int64_t* slots, void* cache,
                                   int64_t block_stride, int bs, int fp8, float kv_inv, hipStream_t st) {
  if (T == 0) return 0;
#define RC(F8)                                                                                                 \
  hipLaunchKernelGGL(mla_rope_cache_kernel<F8>, dim3(T), dim3(256), 0, st, (const uint16_t*)q, q_stride,      \
                     (uint16_t*)q_lat, ql_stride, (const uint16_t*)kv_c, kvc_stride, (const uint16_t*)k_pe,   \
                     kpe_stride, positions, cos_sin, H, slots, cache, block_stride, bs, kv_inv)
  if (fp8) RC(true); else RC(false);
#undef RC
  return (int)hipGetLastError();
}
