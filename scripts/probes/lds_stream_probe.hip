// HBM -> LDS streaming rate vs bytes in flight per CU (decides the MoE v5 pipeline depth).
// 256 workgroups (one per CU, 256 threads = 4 waves), each streams its own contiguous slice of a
// 4 GiB buffer through an S-stage ring of STAGE-byte LDS stages with 16-B LDS-DMA per lane
// (buffer_load_dwordx4 ... lds), keeping S - 1 stages in flight (counted vmcnt + barrier per stage,
// as the GEMM kernels do). Prints GB/s for each (STAGE, S).
//   hipcc --offload-arch=gfx950 -O3 -o lds_stream_probe lds_stream_probe.hip && ./lds_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

template <int STAGE, int S>
__global__ __launch_bounds__(256, 1) void stream_kernel(const uint8_t* __restrict__ src, int64_t per_wg, int* out) {
  __shared__ __attribute__((aligned(1024))) char lds[STAGE * S];
  constexpr int PIECES = STAGE / 1024 / 4;  // 1 KB pieces per wave per stage
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint8_t* base = src + (int64_t)blockIdx.x * per_wg;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  const int nst = (int)(per_wg / STAGE);
  auto issue = [&](int t) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      const uint32_t voff = (uint32_t)((w * PIECES + j) * 1024 + lane * 16);
      char* dst = lds + (t % S) * STAGE + (w * PIECES + j) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff,
                                               (uint32_t)(t * STAGE), 0, 0);
    }
  };
  for (int t = 0; t < S - 1; ++t) issue(t);
  int acc = 0;
  for (int t = 0; t < nst; ++t) {
    if (t + S - 1 < nst) issue(t + S - 1);
    // stage t landed: everything but the newest S - 1 stages
    if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
    if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
    if constexpr (S == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PIECES) : "memory");
    if constexpr (S == 6) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * PIECES) : "memory");
    __builtin_amdgcn_s_barrier();
    acc += *reinterpret_cast<const int*>(lds + (t % S) * STAGE + threadIdx.x * 4);  // touch the stage
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x7fffffff) out[blockIdx.x] = acc;
}

// MoE-like pattern: each workgroup owns a 256-row tile of a [rows, K] row-major matrix and reads,
// per stage, 128 B of every one of its 256 rows (rows `rstride` bytes apart): 32 KB per stage as
// 256 separate 128-B segments (the fp8 grouped GEMM's W stream), vs the contiguous form above.
template <int S>
__global__ __launch_bounds__(256, 1) void strided_kernel(const uint8_t* __restrict__ src, int rstride, int nst,
                                                         int* out) {
  constexpr int STAGE = 32768, PIECES = 8;  // 256 rows x 128 B; 8 pieces (8 rows x 128 B) per wave
  __shared__ __attribute__((aligned(1024))) char lds[STAGE * S];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint8_t* base = src + (int64_t)blockIdx.x * 256 * rstride;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  auto issue = [&](int t) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      const int row = 64 * w + 8 * j + (lane >> 3);
      const uint32_t voff = (uint32_t)(row * rstride + (lane & 7) * 16);
      char* dst = lds + (t % S) * STAGE + (w * PIECES + j) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff,
                                               (uint32_t)(t * 128), 0, 0);
    }
  };
  for (int t = 0; t < S - 1; ++t) issue(t);
  int acc = 0;
  for (int t = 0; t < nst; ++t) {
    if (t + S - 1 < nst) issue(t + S - 1);
    if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    acc += *reinterpret_cast<const int*>(lds + (t % S) * STAGE + threadIdx.x * 4);
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x7fffffff) out[blockIdx.x] = acc;
}

template <int S>
void run_strided(const uint8_t* buf, int rstride, int tiles, int* out) {
  const int nst = rstride / 128;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  strided_kernel<S><<<tiles, 256>>>(buf, rstride, nst, out);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) strided_kernel<S><<<tiles, 256>>>(buf, rstride, nst, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = 5.0 * tiles * 256.0 * rstride;
  printf("strided 256 rows x %5d B (128 B per row per stage) x %d stages, %d tiles: %7.1f GB/s\n", rstride, S, tiles,
         bytes / (ms * 1e-3) / 1e9);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

template <int STAGE, int S>
void run(const uint8_t* buf, int64_t total, int* out) {
  const int64_t per_wg = (total / 256) / STAGE * STAGE;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  stream_kernel<STAGE, S><<<256, 256>>>(buf, per_wg, out);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) stream_kernel<STAGE, S><<<256, 256>>>(buf, per_wg, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double gbs = 5.0 * per_wg * 256 / (ms * 1e-3) / 1e9;
  printf("stage %3d KB x %d stages: in flight ~%3d KB/CU  %7.1f GB/s  (%5.1f GB/s per CU)\n", STAGE / 1024, S,
         STAGE * (S - 1) / 1024, gbs, gbs / 256);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const int64_t total = 4LL << 30;
  uint8_t* buf;
  int* out;
  if (hipMalloc(&buf, total) != hipSuccess || hipMalloc(&out, 256 * sizeof(int)) != hipSuccess) return 1;
  hipMemset(buf, 1, total);
  hipDeviceSynchronize();
  run<16384, 2>(buf, total, out);
  run<16384, 4>(buf, total, out);
  run<16384, 6>(buf, total, out);
  run<32768, 2>(buf, total, out);
  run<32768, 3>(buf, total, out);
  run<32768, 4>(buf, total, out);
  run<49152, 2>(buf, total, out);
  run<49152, 3>(buf, total, out);
  run<65536, 2>(buf, total, out);
  // gpt-oss expert rows: K = 2944 B (2880 padded); 2944 tiles = one grouped GEMM's worth (2.2 GB)
  run_strided<2>(buf, 2944, 2816, out);
  run_strided<3>(buf, 2944, 2816, out);
  run_strided<2>(buf, 8192, 1024, out);
  run_strided<2>(buf, 16384, 512, out);
  hipFree(buf);
  hipFree(out);
  return 0;
}
