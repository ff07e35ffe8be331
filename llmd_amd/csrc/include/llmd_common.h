// Shared device helpers for the llmd_amd HIP op library (gfx950 / CDNA4 only).
//
// Conventions:
//   * bf16 tensors are handled as raw 16-bit words (uint16_t) and widened to
//     f32 with a shift; f32 -> bf16 uses the compiler's __bf16 conversion,
//     which lowers to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving).
//   * All memory-bound kernels move 16 B per lane (8 x bf16) per access.
//   * Wave width is 64 everywhere (hard-coded, never warpSize).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LLMD_WAVE 64

// Device-side invariant checks, compiled in only for the debug op library
// (python -m llmd_amd.build debug -> llmd_amd/_C_debug, loaded when
// LLMD_KERNEL_DEBUG=1): a violated check aborts the kernel with
// file:line instead of faulting on a wild address.
#ifdef LLMD_KERNEL_DEBUG
#include <cassert>
#define LLMD_DCHECK(cond) assert(cond)
#else
#define LLMD_DCHECK(cond) ((void)0)
#endif

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

namespace llmd {

__device__ __forceinline__ float bf2f(uint16_t x) {
  return __uint_as_float(((uint32_t)x) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}
// Unpack a 16-byte chunk of 8 bf16 into 8 floats.
__device__ __forceinline__ void unpack8(const u32x4_t v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4_t pack8(const float* f) {
  u32x4_t v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  }
  return v;
}

// ---- FP8 (OCP e4m3fn on gfx950). KV-cache / activation storage
// format; math stays bf16/f32. Scales are applied outside (folded into the
// softmax scale / output), so conversions here are unscaled.
constexpr float FP8_MAX = 448.f;

// Smallest power of two >= r (r > 0, normal): block scales of the fp8 MoE path
// are powers of two so the grouped GEMM can hand them to the MFMA as E8M0
// exponents (v_mfma_scale_*: scale = 2^(e - 127)) instead of re-scaling block
// partial sums on the VALU. e4m3's relative precision does not depend on the
// binade, so a power-of-two scale only gives up the unused top of [amax, 448].
__device__ __forceinline__ float pow2_ceil(float r) {
  unsigned u = __float_as_uint(r);
  unsigned e = u >> 23;
  if (u & 0x7fffffu) ++e;
  return __uint_as_float(e << 23);
}
// E8M0 exponent byte of a power-of-two float scale.
__device__ __forceinline__ int e8m0_of(float pow2) { return (int)((__float_as_uint(pow2) >> 23) & 0xffu); }

// 8 floats -> 8 e4m3fn bytes (saturating: v_cvt_pk_fp8_f32 alone would map
// |x| > 448 to NaN).
__device__ __forceinline__ u32x2_t f32x8_to_fp8(const float* f) {
  float c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = fminf(fmaxf(f[i], -FP8_MAX), FP8_MAX);
  u32x2_t r;
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  r[0] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  r[1] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
  return r;
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// 8 e4m3fn bytes -> 8 bf16 (exact: every e4m3 value is representable in bf16)
__device__ __forceinline__ u32x4_t fp8x8_to_bf16x8(const u32x2_t v) {
  u32x4_t r;
  r[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v[0], 1.f, false));
  r[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v[0], 1.f, true));
  r[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v[1], 1.f, false));
  r[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v[1], 1.f, true));
  return r;
}

// Load 8 consecutive cache elements as 8 bf16 (16 B), from a bf16 or fp8 cache.
template <bool F8>
__device__ __forceinline__ u32x4_t load8_as_bf16(const void* base, int64_t elem_off) {
  if constexpr (F8) {
    return fp8x8_to_bf16x8(*reinterpret_cast<const u32x2_t*>(reinterpret_cast<const uint8_t*>(base) + elem_off));
  } else {
    return *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint16_t*>(base) + elem_off);
  }
}

// Store 8 bf16 (packed in 16 B) to a bf16 or fp8 cache at element offset;
// fp8 stores multiply by inv_scale first.
template <bool F8>
__device__ __forceinline__ void store8_from_bf16(void* base, int64_t elem_off, const u32x4_t v, float inv_scale) {
  if constexpr (F8) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] *= inv_scale;
    *reinterpret_cast<u32x2_t*>(reinterpret_cast<uint8_t*>(base) + elem_off) = f32x8_to_fp8(f);
  } else {
    *reinterpret_cast<u32x4_t*>(reinterpret_cast<uint16_t*>(base) + elem_off) = v;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// XCD-aware bijective block remap (8 XCDs): consecutive logical tiles land on
// the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// LDS-DMA of one 16-B piece per lane (global_load_lds_dwordx4) written as inline
// asm. A global_load_lds that hipcc can see anywhere in a loop makes its waitcnt
// pass give up on counting LDS reads (every wait becomes lgkmcnt(0), exposing
// each fragment read's latency); issued from asm, the DMA is invisible to it and
// the reads keep counted lgkmcnt(N) waits. The caller waits for the DMA itself
// (s_waitcnt vmcnt(..) before the barrier that publishes the tile): hipcc emits
// no wait for it, and __syncthreads() does not drain it.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
#ifndef LLMD_ASM_DMA
#define LLMD_ASM_DMA 1  // 0: the builtin (hipcc-visible) DMA, for A/B runs
#endif
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
#if !LLMD_ASM_DMA
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)gsrc,
                                   (void __attribute__((address_space(3)))*)(uintptr_t)lds_dst, 16, 0, 0);
  return;
#endif
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

// glds16 with the nt cache policy (a stream read once per launch)
__device__ __forceinline__ void glds16_nt(const void* gsrc, unsigned lds_dst) {
#if !LLMD_ASM_DMA
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)gsrc,
                                   (void __attribute__((address_space(3)))*)(uintptr_t)lds_dst, 16, 0, 2);
  return;
#endif
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

// 4-byte-per-lane form (global_load_lds_dword), same contract as glds16
__device__ __forceinline__ void glds4(const void* gsrc, unsigned lds_dst) {
#if !LLMD_ASM_DMA
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)gsrc,
                                   (void __attribute__((address_space(3)))*)(uintptr_t)lds_dst, 4, 0, 0);
  return;
#endif
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

}  // namespace llmd

#define LLMD_CHECK_LAUNCH() \
  do {                      \
  } while (0)
