// Block-fp8 grouped expert GEMM v8 (the DeepGEMM role; prefill-sized MoE
// steps): the v4 tile loop (moe4.hip moe_gemm4_fp8_kernel: 4 waves, 256 / 192 x 256 tiles,
// scaled 32x32x64 MFMA with the E8M0 block scales as operands, A rows gathered by the
// LDS-DMA) made PERSISTENT so that the per-tile fixed cost is hidden.
//
//   Y[p, :] = X[row(p), :] . W[e(tile)]^T      p = a sorted slot of the tile
//
// Measured (scripts/moe_tile_overhead.py, profiles/moe_gemm_v8_r6.txt): the v4 grid pays
// ~16 us per tile at gpt-oss-120b T=5120 (a 23-step tile is ~54 us) and ~21 us at DeepSeek EP8 -
// workgroup dispatch, metadata loads, the first two K-steps' DMA latency and the epilogue, all
// with the matrix cores idle and no weight bytes streaming. Here
//
// * one workgroup per CU walks a list of (expert M tile, N tile) work items. The list is the
//   real tile count (moe_align's padded total, read on the device) split into 8 contiguous
//   chunks, one per XCD (workgroup b runs on XCD b % 8), so the workgroups of an XCD work on
//   consecutive items: the gathered A rows of an M tile and the weight panel shared by an
//   expert's M tiles are read from HBM once per XCD and served from its L2;
// * the LDS-DMA stream never stops at a tile edge: the K-steps of consecutive tiles form one
//   stream (buffer parity = global step parity), the DMAs issued during a tile's last two steps
//   load the NEXT tile's steps 0 and 1 (descriptors swapped after step nk - 3's DMAs; its
//   metadata - expert id, sorted slots, valid-row count - is loaded at the start of step nk - 3,
//   and its weight scales and bias are DMA'd into the other half of double-buffered LDS slots
//   at step nk - 2). The last step reads the next tile's first fragments, so the next K loop
//   starts without a bubble;
// * the epilogue stores straight from the accumulators (no LDS image: the LDS already holds
//   the next tile's steps). A lane of the 32x32 output layout holds 4 consecutive columns of a
//   row for 4 column groups; one cross-half exchange (lane l <-> l ^ 32) turns them into 16-B
//   row stores. MODE 0: bf16 + expert bias; MODE 1: the gated activation on the interleaved
//   [g0, u0, g1, u1, ..] columns (SiLU or gpt-oss clamped SwiGLU), N / 2 columns stored. Rows
//   past the tile's valid prefix (moe_align pads each expert at its end) are not stored.
//
// The vmcnt accounting of the tile loop is v4's (NPC DMA ops per wave and step, counted waits);
// the extra ops of the tile switch (metadata loads, the weight-scale / bias DMAs of waves 0-1 /
// 2-3, epilogue stores) are always OLDER than the step they precede, so the counted waits only
// become stricter.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int P8_BN = 256, P8_NT = 256;
constexpr int P8_OPB = 256 * 128;  // W bytes per K-step (256 rows x 128 fp8)
constexpr uint32_t P8_OOB = 0x80000000u;

typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void p8_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void p8_mfma(f32x16_t& acc, const i32x8_t& a, const i32x8_t& b, int sa, int sb) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]"
               : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
}

__device__ __forceinline__ void m4b_mfma(f32x4_t& acc, const s16x8_t& a, const s16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// v_rcp_f32 instead of an IEEE divide (~10 VALU ops): the epilogue runs with the MFMA pipe idle, and the
// result is rounded to bf16 anyway
__device__ __forceinline__ float p8_act(float g, float u, int act, float alpha, float limit) {
  if (act == 2) {  // gpt-oss: clamp, (u + 1) * g * sigmoid(alpha * g)
    g = fminf(g, limit);
    u = fminf(fmaxf(u, -limit), limit);
    return (u + 1.f) * g * __builtin_amdgcn_rcpf(1.f + __expf(-alpha * g));
  }
  return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)) * u;
}

__device__ __forceinline__ uint32_t p8_pack(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

template <int MODE, int TBM>
__global__ __launch_bounds__(P8_NT, 1) void moe_gemm8_fp8_kernel(
    const uint8_t* __restrict__ X, int64_t x_stride, const float* __restrict__ xs, int64_t xs_stride, int topk,
    const int* __restrict__ sorted_ids, const int* __restrict__ tile_expert, const int* __restrict__ total_p,
    int max_mtiles, int ntn, int order, const uint8_t* __restrict__ W, int64_t w_expert_stride, const float* __restrict__ ws, int N, int K,
    uint16_t* __restrict__ Y, int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots,
    const uint16_t* __restrict__ bias) {
  static_assert(TBM == 256 || TBM == 192 || TBM == 64, "tile rows");
  constexpr int MB = TBM / 64;                 // 32-row A blocks per wave
  constexpr int NA = 2 * MB;                   // A DMA pieces per wave per K-step
  constexpr int OPA = TBM * 128;               // A bytes per K-step
  constexpr int SCB = TBM * 4 + 256;           // act scales of a K-step (+ the 192 form's overhang)
  constexpr int BUF = OPA + P8_OPB + SCB;
  constexpr int WSO = 2 * BUF;                 // weight scales [2 tile slots][2 col blocks][64 k-blocks] f32
  constexpr int BSO = WSO + 2 * 512;           // bias [2 tile slots][256 columns] bf16
  constexpr int LDSB = BSO + 2 * 512;
  constexpr int NPC = NA + 8 + 1;              // DMA ops per wave per K-step (17 / 15)
  constexpr int NMF = 4 * MB;                  // MFMAs per k-substep
  // schedule slots per half: 64-row tiles (MB = 1: 4 MFMAs per substep, decode-sized steps) run the same
  // op sequence with slots past the last MFMA issuing only their loads / waits / DMAs
  constexpr int T1 = MB == 1 ? 4 + 2 * MB + 3 : NMF;
  constexpr int T2 = MB == 1 ? 12 : NMF;
  constexpr int SROWS = TBM / 4;               // act-scale rows per wave
  constexpr int NQ = TBM / 64;                 // 64-slot groups of a tile (valid-row ballot)
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];  // the ONLY LDS object

  const int nk = K / 128, nnb = (N + 127) / 128;
  // this workgroup's work items: chunk [c0, c1) of XCD x, items c0 + s, c0 + s + S, ...
  const int n_items = min(__builtin_amdgcn_readfirstlane(total_p[0]) / TBM, max_mtiles) * ntn;
  // order 1: items b, b + G, b + 2 G, .. (the v4 grid's order: concurrent items spread over the XCDs)
  const int xcd = blockIdx.x & 7;
  const int S = order ? (int)gridDim.x : (int)(gridDim.x >> 3);
  const int c0 = order ? 0 : (int)((int64_t)n_items * xcd / 8);
  const int c1 = order ? n_items : (int)((int64_t)n_items * (xcd + 1) / 8);
  int item = c0 + (int)(order ? blockIdx.x : blockIdx.x >> 3);
  if (item >= c1) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int l32 = lane & 31, h = lane >> 5;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)xs, 0, 0x7fffffff, 0x00020000);

  // ---- per-tile state (current tile; the next tile's is built at the end of step nk - 3)
  int m0 = 0, n0 = 0, e = 0, nvalid = 0;
  __amdgpu_buffer_rsrc_t rw;
  uint32_t va[8], vw[8], vs;  // fixed-size arrays (a template-sized one can lose the launch stub, build.py)
  int sid_a[8], sid_s, sid_v[4], e_ld;  // a tile's metadata, loaded ahead of build()
  auto meta_load = [&](int it) {
    const int mm = (it / ntn) * TBM;
    e_ld = tile_expert[it / ntn];
#pragma unroll
    for (int j = 0; j < NA; ++j) sid_a[j] = sorted_ids[mm + 8 * (NA * w + j) + (lane >> 3)];
    sid_s = sorted_ids[mm + min(SROWS * w + lane, TBM - 1)];
#pragma unroll
    for (int q = 0; q < NQ; ++q) sid_v[q] = sorted_ids[mm + 64 * q + lane];
  };
  auto build = [&](int it) {
    const int mt = it / ntn;
    m0 = mt * TBM;
    n0 = (it - mt * ntn) * P8_BN;
    e = __builtin_amdgcn_readfirstlane(e_ld);
    int nv = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) nv += __popcll(__ballot(sid_v[q] >= 0));
    nvalid = __builtin_amdgcn_readfirstlane(nv);
    if (e < 0) {  // not a real tile (the item list is the real count; defensive): read zeros, store nothing
      e = 0;
      nvalid = 0;
    }
    rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)e * w_expert_stride), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int row = 8 * (NA * w + j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int sid = sid_a[j];
      const int tok = a_rows_are_slots ? m0 + row : sid / topk;
      va[j] = sid < 0 || nvalid == 0 ? P8_OOB : (uint32_t)((int64_t)tok * x_stride + c * 16);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 64 * w + 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      vw[j] = n0 + row < N ? (uint32_t)((int64_t)(n0 + row) * K + c * 16) : P8_OOB;
    }
    {
      const int row = min(SROWS * w + lane, TBM - 1);
      const int tok = sid_s < 0 ? 0 : (a_rows_are_slots ? m0 + row : sid_s / topk);
      vs = (uint32_t)((int64_t)tok * xs_stride * 4);
    }
  };
  // the tile's weight scales (waves 0 / 1: column blocks n0 / 128 + 0 / 1) and bias (waves 2 / 3:
  // columns n0 + 128 (w - 2) + [0, 128)) into LDS slot `sl`: one extra DMA op for a wave that issues one
  auto side_dma = [&](int sl) {
    if (w < 2) {
      const int cb = min(n0 / 128 + w, nnb - 1);
      const __amdgpu_buffer_rsrc_t rws = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(ws + ((int64_t)e * nnb + cb) * nk), 0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rws, (__attribute__((address_space(3))) void*)(lds + WSO + sl * 512 + w * 256), 4,
          (uint32_t)(min(lane, nk - 1) * 4), 0, 0, 0);
    } else if (bias != nullptr) {
      // 128 bf16 columns = 64 lanes x 4 B; columns past N read zeros (never stored)
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(bias + (int64_t)e * N), 0, (uint32_t)N * 2, 0x00020000);
      const int col = n0 + 128 * (w - 2) + 2 * lane;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(lds + BSO + sl * 512 + (w - 2) * 256), 4,
          (uint32_t)(col * 2), 0, 0, 0);
    }
  };
  auto dma = [&](int bsel, int kc, int j, int op) {  // op 0 = A piece j, 1 = W piece j, 2 = act scales
    char* buf = lds + bsel * BUF;
    if (op == 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf + OPA + P8_OPB + w * SROWS * 4),
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
  const int s_base = OPA + P8_OPB + wr * (TBM / 2) * 4;

  f32x16_t acc[4][MB];  // [W n-block j][A m-block i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < MB; ++i) acc[j][i] = f32x16_t{};
  i32x8_t fw0[4], fa0[MB], fw1[4], fa1[MB];
  int sa[MB], swt;
  float nsf[MB], nwf;

  // ---- prologue of the first tile: metadata, side DMAs into slot 0, stream steps 0 and 1
  meta_load(item);
  build(item);
  int slot = 0;  // LDS slot of the current tile's weight scales / bias
  side_dma(0);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int j = 0; j < NA; ++j) dma(s, s, j, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(s, s, j, 1);
    dma(s, s, 0, 2);
  }
  if constexpr (NPC == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");  // side DMA + step 0 landed
  else if constexpr (NPC == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
  p8_bar();
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

  // one K-step. PH 0: a step of this tile's own stream; 1 (step nk - 3): the next tile's metadata
  // loads first, its descriptors built after this step's (last own) DMAs; 2 (nk - 2): the next
  // tile's weight-scale / bias DMAs, then its step 0; 3 (nk - 1): its step 1, and the step-0
  // fragments / scales read for the next K loop. With no next tile the "next" one is the current
  // one again (harmless reloads into buffers nobody reads): the step has no data-dependent branch.
  int gs = 0;  // global stream step (LDS buffer parity)
  auto step = [&](auto PH_, int kt, int nx) {
    constexpr int PH = decltype(PH_)::value;
    const int bsel = gs & 1;
    const char* cur = lds + bsel * BUF;
    const char* nxt = lds + (bsel ^ 1) * BUF;
    const int kc = PH <= 1 ? kt + 2 : PH - 2;  // stream step kt + 2 (own, or the next tile's 0 / 1)
    if constexpr (PH == 1) meta_load(nx);  // complete by this step's counted wait (older than its DMAs)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < T1; ++t) {
      const int j = t / MB, i = t % MB;
      if (t < NMF) p8_mfma(acc[j][i], fw0[j], fa0[i], swt, sa[i]);
      if (t < 4) {
        fw1[t] = frag(cur + w_base, t, 1);
      } else if (t < 4 + MB) {
        fa1[t - 4] = frag(cur + a_base, t - 4, 1);
      } else if (t == 4 + MB + 1) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        p8_bar();
        if constexpr (PH == 2) side_dma(slot ^ 1);  // older than this step's DMAs
      } else if (t > 4 + MB + 1 && t < 4 + MB + 2 + MB) {
        const int q = t - (4 + MB + 2);
        dma(bsel, kc, 2 * q, 0);
        dma(bsel, kc, 2 * q + 1, 0);
        if (4 + 2 * MB + 2 >= T1 && t == T1 - 1) dma(bsel, kc, 0, 2);  // 192 rows: the act-scale piece
      } else if (t == 4 + 2 * MB + 2) {
        dma(bsel, kc, 0, 2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      const int j = t / MB, i = t % MB;
      if (t < NMF) p8_mfma(acc[j][i], fw1[j], fa1[i], swt, sa[i]);
      if (t < 8) {
        dma(bsel, kc, t, 1);
      } else if (t == 8) {
        if constexpr (NPC == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
        else if constexpr (NPC == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
        p8_bar();
      } else if (t == 9) {
        // the next stream step's raw scales: act from its buffer, weight from this tile's slot or
        // (last step) the next tile's
#pragma unroll
        for (int b = 0; b < MB; ++b) nsf[b] = *reinterpret_cast<const float*>(nxt + s_base + (32 * b + l32) * 4);
        if constexpr (PH == 3) nwf = *reinterpret_cast<const float*>(lds + WSO + (slot ^ 1) * 512 + wc * 256);
        else nwf = *reinterpret_cast<const float*>(lds + WSO + slot * 512 + wc * 256 + (kt + 1) * 4);
        fw0[0] = frag(nxt + w_base, 0, 0);
        if constexpr (MB == 3 || MB == 1) fw0[1] = frag(nxt + w_base, 1, 0);
      } else if constexpr (MB == 4) {
        if (t < 13) {
          fw0[t - 9] = frag(nxt + w_base, t - 9, 0);
        } else if (t < 15) {
          fa0[2 * (t - 13)] = frag(nxt + a_base, 2 * (t - 13), 0);
          fa0[2 * (t - 13) + 1] = frag(nxt + a_base, 2 * (t - 13) + 1, 0);
        }
      } else {
        if (t == 10) {
          fw0[2] = frag(nxt + w_base, 2, 0);
          fw0[3] = frag(nxt + w_base, 3, 0);
        } else if (t == 11) {
#pragma unroll
          for (int b = 0; b < MB; ++b) fa0[b] = frag(nxt + a_base, b, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) sa[b] = e8m0_of(nsf[b]);
    swt = e8m0_of(nwf);
    // the next tile's descriptors: every DMA of this tile's own steps has been issued
    if constexpr (PH == 1) build(nx);
    // drain at the end of every step (asm MFMAs: hipcc does not model their latency)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    ++gs;
  };
  while (true) {
    const int nxt_item = item + S;
    const bool has_next = nxt_item < c1;
    const int nx = has_next ? nxt_item : item;
    // the current tile's epilogue parameters (build() overwrites the state at step nk - 3)
    const int cm0 = m0, cn0 = n0, cnv = nvalid, cslot = slot;
    for (int kt = 0; kt < nk - 3; ++kt) step(std::integral_constant<int, 0>{}, kt, nx);
    step(std::integral_constant<int, 1>{}, nk - 3, nx);
    step(std::integral_constant<int, 2>{}, nk - 2, nx);
    step(std::integral_constant<int, 3>{}, nk - 1, nx);
    __builtin_amdgcn_sched_barrier(0);

    // ---- epilogue of the current tile straight from the accumulators:
    // acc[j][i][4 g + q] = C[m][n], m = wr*TBM/2 + 32 i + l32, n = wc*128 + 32 j + 8 g + 4 h + q
    const int ncol0 = cn0 + wc * 128;
    const char* bl = lds + BSO + cslot * 512 + wc * 256;  // this wave's 128 bias columns (bf16)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float bv[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2_t raw = u32x2_t{0u, 0u};
        if (bias != nullptr) raw = *reinterpret_cast<const u32x2_t*>(bl + (32 * j + 8 * g + 4 * h) * 2);
        bv[g][0] = __uint_as_float(raw[0] << 16);
        bv[g][1] = __uint_as_float(raw[0] & 0xffff0000u);
        bv[g][2] = __uint_as_float(raw[1] << 16);
        bv[g][3] = __uint_as_float(raw[1] & 0xffff0000u);
      }
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int m = wr * (TBM / 2) + 32 * i + l32;
        const bool live = m < cnv;
        uint16_t* yrow = Y + (int64_t)(cm0 + m) * y_stride;
        float v[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[g][q] = acc[j][i][4 * g + q] + bv[g][q];
        if constexpr (MODE == 0) {
#pragma unroll
          for (int gp = 0; gp < 2; ++gp) {
            const uint32_t a0 = p8_pack(v[2 * gp][0], v[2 * gp][1]), a1 = p8_pack(v[2 * gp][2], v[2 * gp][3]);
            const uint32_t b0 = p8_pack(v[2 * gp + 1][0], v[2 * gp + 1][1]);
            const uint32_t b1 = p8_pack(v[2 * gp + 1][2], v[2 * gp + 1][3]);
            // lane h = 0 keeps column group 2 gp (its 4 columns + the partner's 4), h = 1 group 2 gp + 1
            const uint32_t r0 = (uint32_t)__shfl_xor((int)(h ? a0 : b0), 32, 64);
            const uint32_t r1 = (uint32_t)__shfl_xor((int)(h ? a1 : b1), 32, 64);
            const u32x4_t o = h ? u32x4_t{r0, r1, b0, b1} : u32x4_t{a0, a1, r0, r1};
            const int n = ncol0 + 32 * j + 8 * (2 * gp + h);
            if (live && n < N) *reinterpret_cast<u32x4_t*>(yrow + n) = o;
          }
        } else {
          uint32_t o[4];  // o[g]: outputs (n / 2) = wc*64 + 16 j + 4 g + 2 h + {0, 1}
#pragma unroll
          for (int g = 0; g < 4; ++g)
            o[g] = p8_pack(p8_act(v[g][0], v[g][1], act, alpha, limit), p8_act(v[g][2], v[g][3], act, alpha, limit));
          // lane h = 0 keeps outputs 0..7 of the 16 (groups 0, 1), h = 1 outputs 8..15 (groups 2, 3)
          const uint32_t r0 = (uint32_t)__shfl_xor((int)(h ? o[0] : o[2]), 32, 64);
          const uint32_t r1 = (uint32_t)__shfl_xor((int)(h ? o[1] : o[3]), 32, 64);
          const u32x4_t ov = h ? u32x4_t{r0, o[2], r1, o[3]} : u32x4_t{o[0], r0, o[1], r1};
          const int hc = ncol0 / 2 + 16 * j + 8 * h;
          if (live && 2 * hc < N) *reinterpret_cast<u32x4_t*>(yrow + hc) = ov;
        }
      }
    }
    if (!has_next) break;
    item = nxt_item;
    slot ^= 1;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < MB; ++i) acc[j][i] = f32x16_t{};
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 4" ::: "memory");  // accumulator writes -> MFMA srcC
    __builtin_amdgcn_sched_barrier(0);
  }
  // the last tile's dummy DMAs must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}


typedef int i32x4_t __attribute__((ext_vector_type(4)));

// D(32x32) += (W 32x64 e2m1 x 2^(sw-127) per 32-block) . (A 64x32 e4m3 x 2^(sa-127)): MXFP4 weights as the
// MFMA's A operand (cbsz:4 = e2m1, 4 VGPRs), fp8 activations as B
__device__ __forceinline__ void p4_mfma(f32x16_t& acc, const i32x4_t& a, const i32x8_t& b, int sa, int sb) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0] cbsz:4"
               : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
}

template <int N>
__device__ __forceinline__ void p4_vmwait() {
  static_assert(N == 8 || N == 12 || N == 14 || N == 16 || N == 24 || N == 28, "counted waits of the MXFP4 stream");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
}

// MXFP4 form (gpt-oss ships its experts as OCP MXFP4): the fp8 kernel above with e2m1 weights - half
// the weight bytes per K-step (64 B per row: 4 DMA pieces per wave instead of 8) and an E8M0 scale per
// (row, 32-element block) DMA'd with each K-step (one 4-B piece per wave) and handed to the MFMA per
// lane and fragment; activations stay block-fp8 (e4m3, power-of-two (token, 128) scales).
template <int MODE, int TBM, int NS, int DIAG = 0>
__global__ __launch_bounds__(P8_NT, 1) void moe_gemm8_mxfp4_kernel(
    const uint8_t* __restrict__ X, int64_t x_stride, const float* __restrict__ xs, int64_t xs_stride, int topk,
    const int* __restrict__ sorted_ids, const int* __restrict__ tile_expert, const int* __restrict__ total_p,
    int max_mtiles, int ntn, int order, const uint8_t* __restrict__ W, int64_t w_expert_stride,
    const uint8_t* __restrict__ wsc, int64_t wsc_expert_stride, int N, int K,
    uint16_t* __restrict__ Y, int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots,
    const uint16_t* __restrict__ bias, int w_kmajor) {
  static_assert(TBM == 256 || TBM == 192 || TBM == 64, "tile rows");
  static_assert(NS == 2 || NS == 3, "stream depth");
  constexpr int MB = TBM / 64;                 // 32-row A blocks per wave
  constexpr int NA = 2 * MB;                   // A DMA pieces per wave per K-step
  constexpr int OPA = TBM * 128;               // A bytes per K-step
  constexpr int SCB = TBM * 4 + 256;           // act scales of a K-step (+ the 192 form's overhang)
  constexpr int WB = 256 * 64;                 // e2m1 W bytes per K-step (256 rows x 128 codes)
  constexpr int WSB = 256 * 4;                 // E8M0 W scales per K-step (4 per row)
  constexpr int BUF = OPA + WB + WSB + SCB;
  constexpr int BSO = NS * BUF;                // bias [2 tile slots][256 columns] bf16
  constexpr int LDSB = BSO + 2 * 512;
  constexpr int NPC = NA + 4 + 1 + 1;          // DMA ops per wave per K-step: A, W, W scales, act scales (14 / 12)
  constexpr int NMF = 4 * MB;                  // MFMAs per k-substep
  // schedule slots per half: 64-row tiles (MB = 1: 4 MFMAs per substep) run the same op sequence with
  // slots past the last MFMA issuing only their loads / waits / DMAs
  constexpr int T1 = MB == 1 ? 4 + 2 * MB + 3 : NMF;
  constexpr int T2 = MB == 1 ? 12 : NMF;
  constexpr int SROWS = TBM / 4;               // act-scale rows per wave
  constexpr int NQ = TBM / 64;                 // 64-slot groups of a tile (valid-row ballot)
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];  // the ONLY LDS object

  const int nk = K / 128;
  const int wstep = w_kmajor ? N * 64 : 64;  // W bytes between consecutive K-steps of a row
  const int sstep = w_kmajor ? N * 4 : 4;    // and of its E8M0 scales
  // this workgroup's work items: chunk [c0, c1) of XCD x, items c0 + s, c0 + s + S, ...
  const int n_items = min(__builtin_amdgcn_readfirstlane(total_p[0]) / TBM, max_mtiles) * ntn;
  // order 1: items b, b + G, b + 2 G, .. (the v4 grid's order: concurrent items spread over the XCDs)
  const int xcd = blockIdx.x & 7;
  const int S = order ? (int)gridDim.x : (int)(gridDim.x >> 3);
  const int c0 = order ? 0 : (int)((int64_t)n_items * xcd / 8);
  const int c1 = order ? n_items : (int)((int64_t)n_items * (xcd + 1) / 8);
  int item = c0 + (int)(order ? blockIdx.x : blockIdx.x >> 3);
  if (item >= c1) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int l32 = lane & 31, h = lane >> 5;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)xs, 0, 0x7fffffff, 0x00020000);

  // ---- per-tile state (current tile; the next tile's is built at the end of step nk - 3)
  int m0 = 0, n0 = 0, e = 0, nvalid = 0;
  __amdgpu_buffer_rsrc_t rw;
  __amdgpu_buffer_rsrc_t rsw;
  uint32_t va[8], vw[4], vs, vsw;  // fixed-size arrays (a template-sized one can lose the launch stub, build.py)
  int sid_a[8], sid_s, sid_v[4], e_ld;  // a tile's metadata, loaded ahead of build()
  auto meta_load = [&](int it) {
    const int mm = (it / ntn) * TBM;
    e_ld = tile_expert[it / ntn];
#pragma unroll
    for (int j = 0; j < NA; ++j) sid_a[j] = sorted_ids[mm + 8 * (NA * w + j) + (lane >> 3)];
    sid_s = sorted_ids[mm + min(SROWS * w + lane, TBM - 1)];
#pragma unroll
    for (int q = 0; q < NQ; ++q) sid_v[q] = sorted_ids[mm + 64 * q + lane];
  };
  auto build = [&](int it) {
    const int mt = it / ntn;
    m0 = mt * TBM;
    n0 = (it - mt * ntn) * P8_BN;
    e = __builtin_amdgcn_readfirstlane(e_ld);
    int nv = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) nv += __popcll(__ballot(sid_v[q] >= 0));
    nvalid = __builtin_amdgcn_readfirstlane(nv);
    if (e < 0) {  // not a real tile (the item list is the real count; defensive): read zeros, store nothing
      e = 0;
      nvalid = 0;
    }
    rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)e * w_expert_stride), 0, 0x7fffffff, 0x00020000);
    rsw = __builtin_amdgcn_make_buffer_rsrc((void*)(wsc + (int64_t)e * wsc_expert_stride), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int row = 8 * (NA * w + j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int sid = sid_a[j];
      const int tok = a_rows_are_slots ? m0 + row : sid / topk;
      va[j] = sid < 0 || nvalid == 0 ? P8_OOB : (uint32_t)((int64_t)tok * x_stride + c * 16);
    }
    // W piece j of wave w: rows 64 w + 16 j + (lane >> 2), 64-B row = 4 chunks of 16 B, LDS slot
    // lane & 3 <- chunk (lane & 3) ^ ((row >> 2) & 3) (conflict-free 16-row fragment reads)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 64 * w + 16 * j + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      // w_kmajor: W stored [E, K/128, N, 64] (mxfp4_kernel_layout) - a K-step of a 256-row tile is one
      // contiguous 16 KB run instead of 256 half cache lines
      vw[j] = n0 + row < N ? (uint32_t)((int64_t)(n0 + row) * (w_kmajor ? 64 : K / 2) + c * 16) : P8_OOB;
    }
    // W scales: this lane's row 64 w + lane, 4 E8M0 bytes (the K-step's four 32-blocks)
    vsw = n0 + 64 * w + lane < N ? (uint32_t)((int64_t)(n0 + 64 * w + lane) * (w_kmajor ? 4 : K / 32)) : P8_OOB;
    {
      const int row = min(SROWS * w + lane, TBM - 1);
      const int tok = sid_s < 0 ? 0 : (a_rows_are_slots ? m0 + row : sid_s / topk);
      vs = (uint32_t)((int64_t)tok * xs_stride * 4);
    }
  };
  // the tile's bias (waves 2 / 3: columns n0 + 128 (w - 2) + [0, 128)) into LDS slot `sl`
  auto side_dma = [&](int sl) {
    if (w >= 2 && bias != nullptr) {
      // 128 bf16 columns = 64 lanes x 4 B; columns past N read zeros (never stored)
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(bias + (int64_t)e * N), 0, (uint32_t)N * 2, 0x00020000);
      const int col = n0 + 128 * (w - 2) + 2 * lane;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(lds + BSO + sl * 512 + (w - 2) * 256), 4,
          (uint32_t)(col * 2), 0, 0, 0);
    }
  };
  // op 0 = A piece j, 1 = W piece j (< 4), 2 = act scales, 3 = W scales
  auto dma = [&](int bsel, int kc, int j, int op) {
    if constexpr ((DIAG & 2) != 0) return;  // diagnostic: no K-step DMA (LLMD_MXFP4_DIAG)
    if constexpr ((DIAG & 4) != 0) if (op == 0) return;  // diagnostic: no activation (A) pieces
    if constexpr ((DIAG & 8) != 0) if (op == 1) return;  // diagnostic: no weight (W) pieces
    char* buf = lds + bsel * BUF;
    if (op == 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf + OPA + WB + WSB + w * SROWS * 4),
                                               4, vs, (uint32_t)(kc * 4), 0, 0);
    else if (op == 3)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(buf + OPA + WB + w * 256),
                                               4, vsw, (uint32_t)(kc * sstep), 0, 0);
    else if (op == 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(buf + OPA + (4 * w + j) * 1024),
                                               16, vw[j], (uint32_t)(kc * wstep), 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(buf + (NA * w + j) * 1024),
                                               16, va[j], (uint32_t)(kc * 128), 0, 0);
  };
  // fragment of 32-row block b, k-substep s: lane row 32 b + l32, chunks 4 s + 2 h and 4 s + 2 h + 1
  // (e2m1 A operand: lane (row, h) of a 64-deep substep holds K 16h .. 16h+15 and 32+16h .. 32+16h+15 at
  // one scale, measured by scripts/probes/fp4_layout_probe.hip. Feeding a lane the 32 codes of MX block
  // 2s + h in natural order makes the product run over the K permutation that swaps [16, 32) and [32, 48)
  // of every 64; the fp8 activation fragment is read in that same order: chunks 4s + h and 4s + 2 + h.)
  auto frag = [&](const char* base, int b, int s) {
    if constexpr ((DIAG & 1) != 0) return i32x8_t{b, s, 0, 0, 0, 0, 0, 0};  // diagnostic: no fragment reads
    const int row = 32 * b + l32;
    const int f = (row >> 1) & 7;
    const char* rp = base + row * 128;
    const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(rp + (((4 * s + h) ^ f) * 16));
    const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(rp + (((4 * s + 2 + h) ^ f) * 16));
    return i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  // W fragment of 32-row block b, k-substep s: row 32 b + l32 of this wave's 128, 16 B = codes
  // [64 s + 32 h, +32) = chunk 2 s + h; its E8M0 scale: byte 2 s + h of the row's 4
  auto wfrag = [&](const char* base, int b, int s) {
    if constexpr ((DIAG & 1) != 0) return i32x4_t{b, s, 0, 0};
    const int row = 32 * b + l32;
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(base + row * 64 + (((2 * s + h) ^ ((row >> 2) & 3)) * 16));
    return i32x4_t{(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
  };
  auto wscale = [&](const char* base, int b, int s) {
    if constexpr ((DIAG & 1) != 0) return 127;
    return (int)*reinterpret_cast<const uint8_t*>(base + (32 * b + l32) * 4 + 2 * s + h);
  };
  const int a_base = wr * (TBM / 2) * 128, w_base = OPA + wc * 128 * 64, ws_base = OPA + WB + wc * 128 * 4;
  const int s_base = OPA + WB + WSB + wr * (TBM / 2) * 4;

  f32x16_t acc[4][MB];  // [W n-block j][A m-block i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < MB; ++i) acc[j][i] = f32x16_t{};
  i32x4_t fw0[4], fw1[4];
  i32x8_t fa0[MB], fa1[MB];
  int sa[MB], sw0[4], sw1[4];
  float nsf[MB];

  // ---- prologue of the first tile: metadata, side DMAs into slot 0, stream steps 0 and 1
  meta_load(item);
  build(item);
  int slot = 0;  // LDS slot of the current tile's bias
  side_dma(0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int j = 0; j < NA; ++j) dma(s, s, j, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) dma(s, s, j, 1);
    dma(s, s, 0, 2);
    dma(s, s, 0, 3);
  }
  p4_vmwait<(NS - 1) * NPC>();  // side DMA + step 0 landed
  p8_bar();
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    fw0[b] = wfrag(lds + w_base, b, 0);
    sw0[b] = wscale(lds + ws_base, b, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    fa0[b] = frag(lds + a_base, b, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) sa[b] = e8m0_of(*reinterpret_cast<const float*>(lds + s_base + (32 * b + l32) * 4));
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // one K-step. PH 0: a step of this tile's own stream; 1 (step nk - 3): the next tile's metadata
  // loads first, its descriptors built after this step's (last own) DMAs; 2 (nk - 2): the next
  // tile's weight-scale / bias DMAs, then its step 0; 3 (nk - 1): its step 1, and the step-0
  // fragments / scales read for the next K loop. With no next tile the "next" one is the current
  // one again (harmless reloads into buffers nobody reads): the step has no data-dependent branch.
  int bsel = 0;  // LDS buffer of the current stream step (stream step g lives in buffer g % NS)
  auto step = [&](auto PH_, int kt, int nx) {
    constexpr int PH = decltype(PH_)::value;
    const int bnx = bsel + 1 == NS ? 0 : bsel + 1;
    const char* cur = lds + bsel * BUF;
    const char* nxt = lds + bnx * BUF;
    const int kc = PH <= 1 ? kt + NS : PH - 2;  // stream step kt + NS (own, or the next tile's 0 .. NS - 1)
    if constexpr (PH == 1) meta_load(nx);  // complete by this step's counted wait (older than its DMAs)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < T1; ++t) {
      const int j = t / MB, i = t % MB;
      if (t < NMF) p4_mfma(acc[j][i], fw0[j], fa0[i], sw0[j], sa[i]);
      if (t < 4) {
        fw1[t] = wfrag(cur + w_base, t, 1);
        sw1[t] = wscale(cur + ws_base, t, 1);
      } else if (t < 4 + MB) {
        fa1[t - 4] = frag(cur + a_base, t - 4, 1);
      } else if (t == 4 + MB + 1) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        p8_bar();
        if constexpr (PH == 2) side_dma(slot ^ 1);  // older than this step's DMAs
      } else if (t > 4 + MB + 1 && t < 4 + MB + 2 + MB) {
        const int q = t - (4 + MB + 2);
        dma(bsel, kc, 2 * q, 0);
        dma(bsel, kc, 2 * q + 1, 0);
        if (4 + 2 * MB + 2 >= T1 && t == T1 - 1) dma(bsel, kc, 0, 2);  // 192 rows: the act-scale piece
      } else if (t == 4 + 2 * MB + 2) {
        dma(bsel, kc, 0, 2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      const int j = t / MB, i = t % MB;
      if (t < NMF) p4_mfma(acc[j][i], fw1[j], fa1[i], sw1[j], sa[i]);
      if (t < 4) {
        dma(bsel, kc, t, 1);
      } else if (t == 4) {
        dma(bsel, kc, 0, 3);
      } else if (t == 8) {
        // stream step kt + 1 landed (NS - 1 steps stay in flight); the PH 1 step also waits for
        // its metadata loads, which are younger than step kt + 2's DMAs when NS = 3
        p4_vmwait<(PH == 1 ? 1 : NS - 1) * NPC>();
        p8_bar();
      } else if (t == 9) {
        // the next stream step's act scales and its substep-0 W fragments with their scales
#pragma unroll
        for (int b = 0; b < MB; ++b) nsf[b] = *reinterpret_cast<const float*>(nxt + s_base + (32 * b + l32) * 4);
        fw0[0] = wfrag(nxt + w_base, 0, 0);
        sw0[0] = wscale(nxt + ws_base, 0, 0);
        if constexpr (MB == 3 || MB == 1) {
          fw0[1] = wfrag(nxt + w_base, 1, 0);
          sw0[1] = wscale(nxt + ws_base, 1, 0);
        }
      } else if constexpr (MB == 4) {
        if (t < 13) {
          fw0[t - 9] = wfrag(nxt + w_base, t - 9, 0);
          sw0[t - 9] = wscale(nxt + ws_base, t - 9, 0);
        } else if (t < 15) {
          fa0[2 * (t - 13)] = frag(nxt + a_base, 2 * (t - 13), 0);
          fa0[2 * (t - 13) + 1] = frag(nxt + a_base, 2 * (t - 13) + 1, 0);
        }
      } else {
        if (t == 10) {
          fw0[2] = wfrag(nxt + w_base, 2, 0);
          fw0[3] = wfrag(nxt + w_base, 3, 0);
          sw0[2] = wscale(nxt + ws_base, 2, 0);
          sw0[3] = wscale(nxt + ws_base, 3, 0);
        } else if (t == 11) {
#pragma unroll
          for (int b = 0; b < MB; ++b) fa0[b] = frag(nxt + a_base, b, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) sa[b] = e8m0_of(nsf[b]);
    // the next tile's descriptors: every DMA of this tile's own steps has been issued
    if constexpr (PH == 1) build(nx);
    // drain at the end of every step (asm MFMAs: hipcc does not model their latency)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bsel = bnx;
  };
  while (true) {
    const int nxt_item = item + S;
    const bool has_next = nxt_item < c1;
    const int nx = has_next ? nxt_item : item;
    // the current tile's epilogue parameters (build() overwrites the state at step nk - NS - 1)
    const int cm0 = m0, cn0 = n0, cnv = nvalid, cslot = slot;
    for (int kt = 0; kt < nk - NS - 1; ++kt) step(std::integral_constant<int, 0>{}, kt, nx);
    step(std::integral_constant<int, 1>{}, nk - NS - 1, nx);
    step(std::integral_constant<int, 2>{}, nk - NS, nx);
    step(std::integral_constant<int, 3>{}, nk - NS + 1, nx);
    if constexpr (NS == 3) step(std::integral_constant<int, 4>{}, nk - 1, nx);
    __builtin_amdgcn_sched_barrier(0);

    // ---- epilogue of the current tile straight from the accumulators:
    // acc[j][i][4 g + q] = C[m][n], m = wr*TBM/2 + 32 i + l32, n = wc*128 + 32 j + 8 g + 4 h + q
    const int ncol0 = cn0 + wc * 128;
    const char* bl = lds + BSO + cslot * 512 + wc * 256;  // this wave's 128 bias columns (bf16)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float bv[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2_t raw = u32x2_t{0u, 0u};
        if (bias != nullptr) raw = *reinterpret_cast<const u32x2_t*>(bl + (32 * j + 8 * g + 4 * h) * 2);
        bv[g][0] = __uint_as_float(raw[0] << 16);
        bv[g][1] = __uint_as_float(raw[0] & 0xffff0000u);
        bv[g][2] = __uint_as_float(raw[1] << 16);
        bv[g][3] = __uint_as_float(raw[1] & 0xffff0000u);
      }
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int m = wr * (TBM / 2) + 32 * i + l32;
        const bool live = m < cnv;
        uint16_t* yrow = Y + (int64_t)(cm0 + m) * y_stride;
        float v[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[g][q] = acc[j][i][4 * g + q] + bv[g][q];
        if constexpr (MODE == 0) {
#pragma unroll
          for (int gp = 0; gp < 2; ++gp) {
            const uint32_t a0 = p8_pack(v[2 * gp][0], v[2 * gp][1]), a1 = p8_pack(v[2 * gp][2], v[2 * gp][3]);
            const uint32_t b0 = p8_pack(v[2 * gp + 1][0], v[2 * gp + 1][1]);
            const uint32_t b1 = p8_pack(v[2 * gp + 1][2], v[2 * gp + 1][3]);
            // lane h = 0 keeps column group 2 gp (its 4 columns + the partner's 4), h = 1 group 2 gp + 1
            const uint32_t r0 = (uint32_t)__shfl_xor((int)(h ? a0 : b0), 32, 64);
            const uint32_t r1 = (uint32_t)__shfl_xor((int)(h ? a1 : b1), 32, 64);
            const u32x4_t o = h ? u32x4_t{r0, r1, b0, b1} : u32x4_t{a0, a1, r0, r1};
            const int n = ncol0 + 32 * j + 8 * (2 * gp + h);
            if (live && n < N) *reinterpret_cast<u32x4_t*>(yrow + n) = o;
          }
        } else {
          uint32_t o[4];  // o[g]: outputs (n / 2) = wc*64 + 16 j + 4 g + 2 h + {0, 1}
#pragma unroll
          for (int g = 0; g < 4; ++g)
            o[g] = p8_pack(p8_act(v[g][0], v[g][1], act, alpha, limit), p8_act(v[g][2], v[g][3], act, alpha, limit));
          // lane h = 0 keeps outputs 0..7 of the 16 (groups 0, 1), h = 1 outputs 8..15 (groups 2, 3)
          const uint32_t r0 = (uint32_t)__shfl_xor((int)(h ? o[0] : o[2]), 32, 64);
          const uint32_t r1 = (uint32_t)__shfl_xor((int)(h ? o[1] : o[3]), 32, 64);
          const u32x4_t ov = h ? u32x4_t{r0, o[2], r1, o[3]} : u32x4_t{o[0], r0, o[1], r1};
          const int hc = ncol0 / 2 + 16 * j + 8 * h;
          if (live && 2 * hc < N) *reinterpret_cast<u32x4_t*>(yrow + hc) = ov;
        }
      }
    }
    if (!has_next) break;
    item = nxt_item;
    slot ^= 1;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < MB; ++i) acc[j][i] = f32x16_t{};
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 4" ::: "memory");  // accumulator writes -> MFMA srcC
    __builtin_amdgcn_sched_barrier(0);
  }
  // the last tile's dummy DMAs must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}



// bf16 form: the v4 bf16 tile loop (moe4.hip moe_gemm4_bf16_kernel: 16x16x32 bf16 MFMA, 64-deep
// K-steps, MI = TBM / 32 A fragments per wave, NPC = MI + 8 DMA pieces per wave and step) in the
// same persistent frame. No scales; the side DMA is the bias only (waves 2 / 3). Epilogue layout:
// acc[i][j][r] = C[m][n], m = wr*TBM/2 + 16 i + (lane & 15), n = wc*128 + 16 j + 4 (lane >> 4) + r;
// lanes l and l ^ 16 exchange one column group so a lane holds 8 consecutive columns.
template <int MODE, int TBM>
__global__ __launch_bounds__(P8_NT, 1) void moe_gemm8_bf16_kernel(
    const uint16_t* __restrict__ X, int64_t x_stride, int topk, const int* __restrict__ sorted_ids,
    const int* __restrict__ tile_expert, const int* __restrict__ total_p, int max_mtiles, int ntn, int order,
    const uint16_t* __restrict__ W, int64_t w_expert_stride, int N, int K, uint16_t* __restrict__ Y,
    int64_t y_stride, int act, float alpha, float limit, int a_rows_are_slots, const uint16_t* __restrict__ bias) {
  static_assert(TBM == 256 || TBM == 192, "tile rows");
  constexpr int MI = TBM / 32;             // 16-row A fragments per wave (8 / 6)
  constexpr int OPA = TBM * 128;           // A bytes per K-step (64 bf16 per row)
  constexpr int BUF = OPA + P8_OPB;        // A | W of one K-step
  constexpr int BSO = 2 * BUF;             // bias [2 tile slots][256 columns] bf16
  constexpr int LDSB = BSO + 2 * 512;
  constexpr int NPC = MI + 8;              // DMA pieces per wave per K-step (= fragment reads per half)
  constexpr int NMF = 8 * MI;              // MFMAs per half
  constexpr int TB = 8 * MI - 24;          // half 0: barrier MFMA index (A pieces of step kt + 2 after it)
  constexpr int WP = MI == 8 ? 5 : 4;      // half 1: one W piece every WP MFMAs
  constexpr int RB = MI == 8 ? 37 : 30;    // half 1: first next-step read
  constexpr int NQ = TBM / 64;
  static_assert(TB + 1 + 3 * (MI - 1) < NMF && 8 + MI <= TB && 7 * WP < RB - 1 && RB + NPC <= NMF, "schedule");
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];  // the ONLY LDS object

  const int nk = K / 64;
  const int n_items = min(__builtin_amdgcn_readfirstlane(total_p[0]) / TBM, max_mtiles) * ntn;
  const int xcd = blockIdx.x & 7;
  const int S = order ? (int)gridDim.x : (int)(gridDim.x >> 3);
  const int c0 = order ? 0 : (int)((int64_t)n_items * xcd / 8);
  const int c1 = order ? n_items : (int)((int64_t)n_items * (xcd + 1) / 8);
  int item = c0 + (int)(order ? blockIdx.x : blockIdx.x >> 3);
  if (item >= c1) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, 0x7fffffff, 0x00020000);

  int m0 = 0, n0 = 0, e = 0, nvalid = 0;
  __amdgpu_buffer_rsrc_t rw;
  uint32_t va[8], vw[8];
  int sid_a[8], sid_v[4], e_ld;
  auto meta_load = [&](int it) {
    const int mm = (it / ntn) * TBM;
    e_ld = tile_expert[it / ntn];
#pragma unroll
    for (int j = 0; j < MI; ++j) sid_a[j] = sorted_ids[mm + 8 * (MI * w + j) + (lane >> 3)];
#pragma unroll
    for (int q = 0; q < NQ; ++q) sid_v[q] = sorted_ids[mm + 64 * q + lane];
  };
  auto build = [&](int it) {
    const int mt = it / ntn;
    m0 = mt * TBM;
    n0 = (it - mt * ntn) * P8_BN;
    e = __builtin_amdgcn_readfirstlane(e_ld);
    int nv = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) nv += __popcll(__ballot(sid_v[q] >= 0));
    nvalid = __builtin_amdgcn_readfirstlane(nv);
    if (e < 0) {
      e = 0;
      nvalid = 0;
    }
    rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)e * w_expert_stride), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < MI; ++j) {
      const int row = 8 * (MI * w + j) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int sid = sid_a[j];
      const int tok = a_rows_are_slots ? m0 + row : sid / topk;
      va[j] = sid < 0 || nvalid == 0 ? P8_OOB : (uint32_t)(((int64_t)tok * x_stride + c * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 64 * w + 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      vw[j] = n0 + row < N ? (uint32_t)(((int64_t)(n0 + row) * K + c * 8) * 2) : P8_OOB;
    }
  };
  auto side_dma = [&](int sl) {  // bias columns n0 + 128 (w - 2) + [0, 128) (waves 2 / 3)
    if (w >= 2 && bias != nullptr) {
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(bias + (int64_t)e * N), 0, (uint32_t)N * 2, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(lds + BSO + sl * 512 + (w - 2) * 256), 4,
          (uint32_t)((n0 + 128 * (w - 2) + 2 * lane) * 2), 0, 0, 0);
    }
  };
  auto dma = [&](int bsel, int kc, int j, bool wop) {
    char* dst = lds + bsel * BUF + (wop ? OPA + (8 * w + j) * 1024 : (MI * w + j) * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wop ? rw : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             wop ? vw[j] : va[j], (uint32_t)(kc * 128), 0, 0);
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

  meta_load(item);
  build(item);
  int slot = 0;
  side_dma(0);
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int j = 0; j < MI; ++j) dma(s2, s2, j, false);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(s2, s2, j, true);
  }
  if constexpr (NPC == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  p8_bar();
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
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  int gs = 0;
  auto step = [&](auto PH_, int kt, int nx) {
    constexpr int PH = decltype(PH_)::value;  // as the fp8 form
    const int bsel = gs & 1;
    const char* cur = lds + bsel * BUF;
    const char* nxt = lds + (bsel ^ 1) * BUF;
    const int kc = PH <= 1 ? kt + 2 : PH - 2;
    if constexpr (PH == 1) meta_load(nx);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NMF; ++t) {
      const int i = t >> 3, j = t & 7;
      if (t <= 8) __builtin_amdgcn_s_waitcnt(0xC07F | ((NPC - 2) << 8));
      m4b_mfma(acc[i][j], fw0[j], fa0[i]);
      if (t == 0) {
        fa1[0] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + rd1);
      } else if (t < 9) {
        fw1[t - 1] = *reinterpret_cast<const s16x8_t*>(cur + w_rd + (t - 1) * 2048 + rd1);
      } else if (t < 8 + MI) {
        fa1[t - 8] = *reinterpret_cast<const s16x8_t*>(cur + a_rd + (t - 8) * 2048 + rd1);
      } else if (t == TB) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        p8_bar();
        if constexpr (PH == 2) side_dma(slot ^ 1);  // older than this step's DMAs
      } else if (t > TB && (t - TB - 1) % 3 == 0 && (t - TB - 1) / 3 < MI) {
        dma(bsel, kc, (t - TB - 1) / 3, false);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < NMF; ++t) {
      const int i = t >> 3, j = t & 7;
      m4b_mfma(acc[i][j], fw1[j], fa1[i]);
      if (t < 8 * WP && t % WP == 0) {
        dma(bsel, kc, t / WP, true);
      } else if (t == RB - 1) {
        if constexpr (NPC == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        p8_bar();
      } else if (t == RB) {
        fa0[0] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + rd0);
      } else if (t > RB && t < RB + 9) {
        fw0[t - RB - 1] = *reinterpret_cast<const s16x8_t*>(nxt + w_rd + (t - RB - 1) * 2048 + rd0);
      } else if (t >= RB + 9 && t < RB + 8 + MI) {
        fa0[t - RB - 8] = *reinterpret_cast<const s16x8_t*>(nxt + a_rd + (t - RB - 8) * 2048 + rd0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PH == 1) build(nx);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    ++gs;
  };
  while (true) {
    const int nxt_item = item + S;
    const bool has_next = nxt_item < c1;
    const int nx = has_next ? nxt_item : item;
    const int cm0 = m0, cn0 = n0, cnv = nvalid, cslot = slot;
    for (int kt = 0; kt < nk - 3; ++kt) step(std::integral_constant<int, 0>{}, kt, nx);
    step(std::integral_constant<int, 1>{}, nk - 3, nx);
    step(std::integral_constant<int, 2>{}, nk - 2, nx);
    step(std::integral_constant<int, 3>{}, nk - 1, nx);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    const int ncol0 = cn0 + wc * 128;
    const char* bl = lds + BSO + cslot * 512 + wc * 256;
    const int odd = fq & 1;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      float bv[2][4];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x2_t raw = u32x2_t{0u, 0u};
        if (bias != nullptr) raw = *reinterpret_cast<const u32x2_t*>(bl + (32 * jp + 16 * s2 + 4 * fq) * 2);
        bv[s2][0] = __uint_as_float(raw[0] << 16);
        bv[s2][1] = __uint_as_float(raw[0] & 0xffff0000u);
        bv[s2][2] = __uint_as_float(raw[1] << 16);
        bv[s2][3] = __uint_as_float(raw[1] & 0xffff0000u);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = wr * (TBM / 2) + 16 * i + fr;
        const bool live = m < cnv;
        uint16_t* yrow = Y + (int64_t)(cm0 + m) * y_stride;
        float v0[4], v1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v0[r] = acc[i][2 * jp][r] + bv[0][r];
          v1[r] = acc[i][2 * jp + 1][r] + bv[1][r];
        }
        if constexpr (MODE == 0) {
          const uint32_t a0 = p8_pack(v0[0], v0[1]), a1 = p8_pack(v0[2], v0[3]);
          const uint32_t b0 = p8_pack(v1[0], v1[1]), b1 = p8_pack(v1[2], v1[3]);
          // even fq keeps column block 2 jp (its 4 columns + the partner's 4), odd fq block 2 jp + 1
          const uint32_t r0 = (uint32_t)__shfl_xor((int)(odd ? a0 : b0), 16, 64);
          const uint32_t r1 = (uint32_t)__shfl_xor((int)(odd ? a1 : b1), 16, 64);
          const u32x4_t o = odd ? u32x4_t{r0, r1, b0, b1} : u32x4_t{a0, a1, r0, r1};
          const int n = ncol0 + 16 * (2 * jp + odd) + 4 * (fq - odd);
          if (live && n < N) *reinterpret_cast<u32x4_t*>(yrow + n) = o;
        } else {
          const uint32_t oa = p8_pack(p8_act(v0[0], v0[1], act, alpha, limit), p8_act(v0[2], v0[3], act, alpha, limit));
          const uint32_t ob = p8_pack(p8_act(v1[0], v1[1], act, alpha, limit), p8_act(v1[2], v1[3], act, alpha, limit));
          const uint32_t r = (uint32_t)__shfl_xor((int)(odd ? oa : ob), 16, 64);
          const u32x2_t o = odd ? u32x2_t{r, ob} : u32x2_t{oa, r};
          const int hc = ncol0 / 2 + 8 * (2 * jp + odd) + 2 * (fq - odd);
          if (live && 2 * hc < N) *reinterpret_cast<u32x2_t*>(yrow + hc) = o;
        }
      }
    }
    if (!has_next) break;
    item = nxt_item;
    slot ^= 1;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 4" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace


namespace {
int p8_cus() {
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8)
      return 256;
    return n;
  }();
  return n_cu;
}
int p8_order() {  // work-item order (LLMD_MOE8_ORDER: 0 XCD chunks, 1 round-robin)
  static const int order = [] {
    const char* v = getenv("LLMD_MOE8_ORDER");
    return v ? atoi(v) : 0;
  }();
  return order;
}
}  // namespace

// Same operands as llmd_moe_gemm4_fp8 (moe4.hip) plus total_p: moe_align's padded slot total on
// the device (the real tile count; num_tiles is only the host-side upper bound). K / 128 >= 4.
extern "C" int llmd_moe_gemm8_fp8(const void* X, int64_t x_stride, const float* xs, int64_t xs_stride, int topk,
                                  const int* sorted_ids, const int* tile_expert, const int* total_p, int num_tiles,
                                  const void* W, int64_t w_expert_stride, const float* ws, int N, int K, void* Y,
                                  int64_t y_stride, int mode, int act, float alpha, float limit,
                                  int a_rows_are_slots, const void* bias, int64_t x_rows, int tile_m,
                                  hipStream_t st) {
  if (K % 128 || K / 128 > 64 || K / 128 < 4 || x_stride % 16 || w_expert_stride % 16 || N % 8 ||
      (mode == 1 && N % 16) || y_stride % 8 || total_p == nullptr)
    return -1;
  if (tile_m != 256 && tile_m != 192 && tile_m != 64) return -1;
  if (x_rows * x_stride + K > 0x7fffffffLL || (int64_t)N * K > 0x7fffffffLL || x_rows * xs_stride * 4 > 0x7fffffffLL)
    return -2;
  if (num_tiles == 0) return 0;
  const int n_cu = p8_cus();
  const int order = p8_order();
  const int ntn = (N + P8_BN - 1) / P8_BN;
  const int64_t upper = (int64_t)num_tiles * ntn;
  const int grid = (int)std::min<int64_t>(n_cu / 8 * 8, (upper + 7) / 8 * 8);  // a multiple of 8 (XCDs)
#define P8_LAUNCH(MODE_, TBM_)                                                                                     \
  hipLaunchKernelGGL((moe_gemm8_fp8_kernel<MODE_, TBM_>), dim3(grid), dim3(P8_NT), 0, st, (const uint8_t*)X,       \
                     x_stride, xs, xs_stride, topk, sorted_ids, tile_expert, total_p, num_tiles, ntn, order,            \
                     (const uint8_t*)W,                                                                            \
                     w_expert_stride, ws, N, K, (uint16_t*)Y, y_stride, act, alpha, limit, a_rows_are_slots,       \
                     (const uint16_t*)bias)
  if (tile_m == 256) {
    if (mode == 0) P8_LAUNCH(0, 256); else P8_LAUNCH(1, 256);
  } else if (tile_m == 192) {
    if (mode == 0) P8_LAUNCH(0, 192); else P8_LAUNCH(1, 192);
  } else {
    if (mode == 0) P8_LAUNCH(0, 64); else P8_LAUNCH(1, 64);
  }
#undef P8_LAUNCH
  return (int)hipGetLastError();
}

// Same operands as llmd_moe_gemm4_bf16 (moe4.hip) plus total_p (see above). K % 64 == 0, K / 64 >= 4.
extern "C" int llmd_moe_gemm8_bf16(const void* X, int64_t x_stride, int topk, const int* sorted_ids,
                                   const int* tile_expert, const int* total_p, int num_tiles, const void* W,
                                   int64_t w_expert_stride, int N, int K, void* Y, int64_t y_stride, int mode, int act,
                                   float alpha, float limit, int a_rows_are_slots, const void* bias, int64_t x_rows,
                                   int tile_m, hipStream_t st) {
  if (K % 64 || K / 64 < 4 || x_stride % 8 || w_expert_stride % 8 || N % 8 || (mode == 1 && N % 16) ||
      y_stride % 8 || total_p == nullptr)
    return -1;
  if (tile_m != 256 && tile_m != 192) return -1;
  if ((x_rows * x_stride + K) * 2 > 0x7fffffffLL || ((int64_t)N * K) * 2 > 0x7fffffffLL) return -2;
  if (num_tiles == 0) return 0;
  const int ntn = (N + P8_BN - 1) / P8_BN;
  const int64_t upper = (int64_t)num_tiles * ntn;
  const int grid = (int)std::min<int64_t>(p8_cus() / 8 * 8, (upper + 7) / 8 * 8);
  const int order = p8_order();
#define P8B_LAUNCH(MODE_, TBM_)                                                                                    \
  hipLaunchKernelGGL((moe_gemm8_bf16_kernel<MODE_, TBM_>), dim3(grid), dim3(P8_NT), 0, st, (const uint16_t*)X,     \
                     x_stride, topk, sorted_ids, tile_expert, total_p, num_tiles, ntn, order, (const uint16_t*)W, \
                     w_expert_stride, N, K, (uint16_t*)Y, y_stride, act, alpha, limit, a_rows_are_slots,          \
                     (const uint16_t*)bias)
  if (tile_m == 256) {
    if (mode == 0) P8B_LAUNCH(0, 256); else P8B_LAUNCH(1, 256);
  } else {
    if (mode == 0) P8B_LAUNCH(0, 192); else P8B_LAUNCH(1, 192);
  }
#undef P8B_LAUNCH
  return (int)hipGetLastError();
}

// MXFP4 experts: X [rows, K] e4m3 with xs [rows, K / 128] power-of-two scales, W [E, N, K / 2] packed
// e2m1 (element 2i in the low nibble), wsc [E, N, K / 32] E8M0. K % 128 == 0, K / 128 >= 4.
extern "C" int llmd_moe_gemm8_mxfp4(const void* X, int64_t x_stride, const float* xs, int64_t xs_stride, int topk,
                                    const int* sorted_ids, const int* tile_expert, const int* total_p, int num_tiles,
                                    const void* W, int64_t w_expert_stride, const void* wsc, int64_t wsc_expert_stride,
                                    int N, int K, void* Y, int64_t y_stride, int mode, int act, float alpha,
                                    float limit, int a_rows_are_slots, const void* bias, int64_t x_rows, int tile_m,
                                    int w_kmajor, hipStream_t st) {
  if (K % 128 || K / 128 < 4 || x_stride % 16 || w_expert_stride % 16 || wsc_expert_stride % 4 || N % 8 ||
      (mode == 1 && N % 16) || y_stride % 8 || total_p == nullptr)
    return -1;
  if (tile_m != 256 && tile_m != 192 && tile_m != 64) return -1;
  if (x_rows * x_stride + K > 0x7fffffffLL || (int64_t)N * K / 2 > 0x7fffffffLL || x_rows * xs_stride * 4 > 0x7fffffffLL)
    return -2;
  if (num_tiles == 0) return 0;
  const int ntn = (N + P8_BN - 1) / P8_BN;
  const int64_t upper = (int64_t)num_tiles * ntn;
  // 64-row tiles fit two workgroups per CU (116 VGPRs + 64 AGPRs, 53 KB LDS): LLMD_MXFP4_WG64 per CU
  const char* wgv = getenv("LLMD_MXFP4_WG64");
  const int per_cu = tile_m == 64 ? (wgv && atoi(wgv) == 1 ? 1 : 2) : 1;
  const int grid = (int)std::min<int64_t>(p8_cus() * per_cu / 8 * 8, (upper + 7) / 8 * 8);
  const int order = p8_order();
  // stream depth: 2 LDS K-step buffers (the fp8 kernel's); LLMD_MXFP4_STAGES=3 takes 3 (e2m1 weights
  // leave room: 3 x 50 KB at 256 rows) - measured equal at every gpt-oss step size, so the K-step is
  // not bound by DMA latency (profiles/moe_mxfp4_r6.txt). Read per launch (tests switch it in-process).
  const char* nsv = getenv("LLMD_MXFP4_STAGES");
  const int ns = nsv && atoi(nsv) == 3 ? 3 : 2;
#define P4_LAUNCH(MODE_, TBM_)                                                                                      \
  do {                                                                                                              \
    if (ns == 3) P4_LAUNCH_NS(MODE_, TBM_, 3); else P4_LAUNCH_NS(MODE_, TBM_, 2);                                   \
  } while (0)
#define P4_LAUNCH_NS(MODE_, TBM_, NS_)                                                                              \
  hipLaunchKernelGGL((moe_gemm8_mxfp4_kernel<MODE_, TBM_, NS_>), dim3(grid), dim3(P8_NT), 0, st, (const uint8_t*)X,      \
                     x_stride, xs, xs_stride, topk, sorted_ids, tile_expert, total_p, num_tiles, ntn, order,         \
                     (const uint8_t*)W, w_expert_stride, (const uint8_t*)wsc, wsc_expert_stride, N, K, (uint16_t*)Y, \
                     y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias, w_kmajor)
  // diagnostic variants (192-row tiles, 2 buffers; outputs are garbage): LLMD_MXFP4_DIAG = 1 no fragment
  // reads, 2 no K-step DMAs, 3 neither, 4 no activation pieces, 8 no weight pieces - what is left of a
  // step without each resource
  const char* dgv = getenv("LLMD_MXFP4_DIAG");
  const int diag = dgv ? atoi(dgv) : 0;
#define P4_DIAG(MODE_, D_)                                                                                          \
  hipLaunchKernelGGL((moe_gemm8_mxfp4_kernel<MODE_, 192, 2, D_>), dim3(grid), dim3(P8_NT), 0, st, (const uint8_t*)X, \
                     x_stride, xs, xs_stride, topk, sorted_ids, tile_expert, total_p, num_tiles, ntn, order,         \
                     (const uint8_t*)W, w_expert_stride, (const uint8_t*)wsc, wsc_expert_stride, N, K, (uint16_t*)Y, \
                     y_stride, act, alpha, limit, a_rows_are_slots, (const uint16_t*)bias, w_kmajor)
  if ((diag == 1 || diag == 2 || diag == 3 || diag == 4 || diag == 8) && tile_m == 192) {
    if (mode == 0) {
      if (diag == 1) P4_DIAG(0, 1); else if (diag == 2) P4_DIAG(0, 2); else if (diag == 3) P4_DIAG(0, 3);
      else if (diag == 4) P4_DIAG(0, 4); else P4_DIAG(0, 8);
    } else {
      if (diag == 1) P4_DIAG(1, 1); else if (diag == 2) P4_DIAG(1, 2); else if (diag == 3) P4_DIAG(1, 3);
      else if (diag == 4) P4_DIAG(1, 4); else P4_DIAG(1, 8);
    }
  } else if (tile_m == 256) {
    if (mode == 0) P4_LAUNCH(0, 256); else P4_LAUNCH(1, 256);
  } else if (tile_m == 192) {
    if (mode == 0) P4_LAUNCH(0, 192); else P4_LAUNCH(1, 192);
  } else {
    if (mode == 0) P4_LAUNCH(0, 64); else P4_LAUNCH(1, 64);
  }
#undef P4_DIAG
#undef P4_LAUNCH
#undef P4_LAUNCH_NS
  return (int)hipGetLastError();
}
