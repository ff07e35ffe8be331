// Probe: sustained rate of v_mfma_scale_f32_32x32x64_f8f6f4 by operand format (the instruction the
// MoE tile kernels issue) next to the bf16 32x32x16 MFMA. Every wave keeps random fragments and 4
// independent accumulators in registers and issues MFMAs back to back, 4 waves per CU on every CU;
// the rate is FLOPs / wall time of one launch (hipEvent), after a warm-up launch.
//   fmt 0: e4m3 x e4m3 (cbsz:0 blgp:0) 1: e2m1 A x e4m3 B (cbsz:4, moe8.hip's MXFP4 kernel)
//       2: e2m1 x e2m1 (cbsz:4 blgp:4) 3: bf16 v_mfma_f32_32x32x16_bf16
// hipcc --offload-arch=gfx950 -O3 scripts/probes/mfma_rate_probe.hip -o scripts/probes/mfma_rate_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <int FMT>
__global__ __launch_bounds__(256, 1) void burn(float* out, int iters) {
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
  i32x8 a, b;
  for (int r = 0; r < 8; ++r) {
    // e4m3 / e2m1 / bf16 bit patterns with the exponent field kept finite (0x77 / 0x3f masks)
    a[r] = (int)(hash32(tid * 16 + r) & 0x77777777u);
    b[r] = (int)(hash32(tid * 16 + 8 + r) & 0x77777777u);
  }
  const i32x4 a4 = {a[0], a[1], a[2], a[3]}, b4 = {b[0], b[1], b[2], b[3]};
  const s16x8 a16 = {(short)(a[0] & 0x3fff), (short)(a[1] & 0x3fff), (short)(a[2] & 0x3fff), (short)(a[3] & 0x3fff),
                     (short)(a[4] & 0x3fff), (short)(a[5] & 0x3fff), (short)(a[6] & 0x3fff), (short)(a[7] & 0x3fff)};
  const s16x8 b16 = {(short)(b[0] & 0x3fff), (short)(b[1] & 0x3fff), (short)(b[2] & 0x3fff), (short)(b[3] & 0x3fff),
                     (short)(b[4] & 0x3fff), (short)(b[5] & 0x3fff), (short)(b[6] & 0x3fff), (short)(b[7] & 0x3fff)};
  const int s = 127;
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    if constexpr (FMT == 0) {
      asm volatile(
          "v_mfma_scale_f32_32x32x64_f8f6f4 %0, %4, %5, %0, %6, %6 op_sel_hi:[0,0,0]\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %1, %4, %5, %1, %6, %6 op_sel_hi:[0,0,0]\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %2, %4, %5, %2, %6, %6 op_sel_hi:[0,0,0]\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %3, %4, %5, %3, %6, %6 op_sel_hi:[0,0,0]"
          : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3) : "v"(a), "v"(b), "v"(s));
    } else if constexpr (FMT == 1) {
      asm volatile(
          "v_mfma_scale_f32_32x32x64_f8f6f4 %0, %4, %5, %0, %6, %6 op_sel_hi:[0,0,0] cbsz:4\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %1, %4, %5, %1, %6, %6 op_sel_hi:[0,0,0] cbsz:4\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %2, %4, %5, %2, %6, %6 op_sel_hi:[0,0,0] cbsz:4\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %3, %4, %5, %3, %6, %6 op_sel_hi:[0,0,0] cbsz:4"
          : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3) : "v"(a4), "v"(b), "v"(s));
    } else if constexpr (FMT == 2) {
      asm volatile(
          "v_mfma_scale_f32_32x32x64_f8f6f4 %0, %4, %5, %0, %6, %6 op_sel_hi:[0,0,0] cbsz:4 blgp:4\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %1, %4, %5, %1, %6, %6 op_sel_hi:[0,0,0] cbsz:4 blgp:4\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %2, %4, %5, %2, %6, %6 op_sel_hi:[0,0,0] cbsz:4 blgp:4\n\t"
          "v_mfma_scale_f32_32x32x64_f8f6f4 %3, %4, %5, %3, %6, %6 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
          : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3) : "v"(a4), "v"(b4), "v"(s));
    } else {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a16, b16, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a16, b16, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a16, b16, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a16, b16, c3, 0, 0, 0);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  float sum = 0.f;
  for (int r = 0; r < 16; ++r) sum += c0[r] + c1[r] + c2[r] + c3[r];
  out[tid] = sum;  // keeps the loop live
}

template <int FMT>
double run(float* out, int cus, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(burn<FMT>, dim3(cus), dim3(256), 0, 0, out, iters / 10);
  hipEventRecord(e0);
  hipLaunchKernelGGL(burn<FMT>, dim3(cus), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double k = FMT == 3 ? 16.0 : 64.0;
  const double flops = (double)cus * 4 * iters * 4 * (2.0 * 32 * 32 * k);
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  float* out;
  hipMalloc(&out, (size_t)cus * 256 * sizeof(float));
  const int iters = 20000;
  printf("CUs %d, 4 waves per CU, 4 independent 32x32 accumulators per wave\n", cus);
  printf("e4m3 x e4m3   32x32x64 scaled: %7.0f TFLOP/s\n", run<0>(out, cus, iters));
  printf("e2m1 x e4m3   32x32x64 scaled: %7.0f TFLOP/s (moe8 MXFP4 kernel's operands)\n", run<1>(out, cus, iters));
  printf("e2m1 x e2m1   32x32x64 scaled: %7.0f TFLOP/s\n", run<2>(out, cus, iters));
  printf("bf16          32x32x16       : %7.0f TFLOP/s\n", run<3>(out, cus, iters));
  hipFree(out);
  return 0;
}
