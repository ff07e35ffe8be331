// kvx: KV-block transfer kernels + IPC helpers (the
// NIXL/RIXL data plane re-done for one xGMI-connected MI355X node).
//
// The decode engine maps the prefill engine's whole KV pool once through a
// HIP IPC handle (peer memory over xGMI, or the same device), then pulls a
// request's blocks with one launch: every workgroup moves 16-byte vectors of
// one (block pair, segment) with non-temporal stores, so the copy streams at
// link rate without polluting the decoder's L2. Segments express layout
// conversion between the two pools, e.g. heterogeneous TP (P holds 8 KV heads
// per block, D rank r takes heads [2r, 2r+2)): for every (layer, K/V plane)
// one segment = (src offset, dst offset, length).
#include <cstring>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;

// pairs[2*i] = src block, pairs[2*i+1] = dst block.
// segs[3*j] = src byte offset in block, segs[3*j+1] = dst byte offset, segs[3*j+2] = bytes (multiple of 16)
__global__ __launch_bounds__(NT) void copy_blocks_kernel(char* __restrict__ dst, const char* __restrict__ src,
                                                         int64_t dst_stride, int64_t src_stride,
                                                         const int* __restrict__ pairs,
                                                         const int64_t* __restrict__ segs, int nseg,
                                                         int64_t chunk_bytes) {
  const int pi = blockIdx.y;
  const int sj = blockIdx.z;
  const int64_t sb = pairs[2 * pi], db = pairs[2 * pi + 1];
  const int64_t so = segs[3 * sj], dof = segs[3 * sj + 1], len = segs[3 * sj + 2];
  const int64_t c0 = (int64_t)blockIdx.x * chunk_bytes;
  if (c0 >= len) return;
  const int64_t c1 = min(len, c0 + chunk_bytes);
  const u32x4_t* s = reinterpret_cast<const u32x4_t*>(src + sb * src_stride + so);
  u32x4_t* d = reinterpret_cast<u32x4_t*>(dst + db * dst_stride + dof);
  const int64_t v0 = c0 / 16, v1 = c1 / 16;
  // 4 independent 16-B loads in flight per lane
  int64_t v = v0 + threadIdx.x;
  for (; v + 3 * NT < v1; v += 4 * NT) {
    u32x4_t a = s[v], b = s[v + NT], c = s[v + 2 * NT], e = s[v + 3 * NT];
    __builtin_nontemporal_store(a, d + v);
    __builtin_nontemporal_store(b, d + v + NT);
    __builtin_nontemporal_store(c, d + v + 2 * NT);
    __builtin_nontemporal_store(e, d + v + 3 * NT);
  }
  for (; v < v1; v += NT) __builtin_nontemporal_store(s[v], d + v);
}

constexpr int CP_NT = 256, CP_CHUNK = 65536;  // 4 waves x 16 KB

__device__ __forceinline__ void cp_dma16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

__global__ __launch_bounds__(CP_NT) void copy_blocks_lds_kernel(char* __restrict__ dst, const char* __restrict__ src,
                                                                int64_t dst_stride, int64_t src_stride,
                                                                const int* __restrict__ pairs,
                                                                const int64_t* __restrict__ segs) {
  __shared__ __attribute__((aligned(1024))) char lds[CP_CHUNK];
  const int pi = blockIdx.y, sj = blockIdx.z;
  const int64_t sb = pairs[2 * pi], db = pairs[2 * pi + 1];
  const int64_t so = segs[3 * sj], dof = segs[3 * sj + 1], len = segs[3 * sj + 2];
  const int64_t c0 = (int64_t)blockIdx.x * CP_CHUNK;
  if (c0 >= len) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t wb = c0 + w * 16384;  // this wave's 16 KB: 16 pieces of 64 lanes x 16 B
  const char* s = src + sb * src_stride + so;
  char* d = dst + db * dst_stride + dof;
  char* lw = lds + w * 16384;         // lane-linear image: piece i at lw + i * 1024
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t off = wb + i * 1024 + lane * 16;
    if (off < len) cp_dma16(s + off, lw + i * 1024);
  }
  // a wave reads back only what its own DMAs wrote: its vmcnt alone orders the reads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t off = wb + i * 1024 + lane * 16;
    if (off < len) {
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(lw + i * 1024 + lane * 16);
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(d + off));
    }
  }
}

}  // namespace

extern "C" {

int llmd_kvx_copy_blocks(void* dst, const void* src, int64_t dst_stride, int64_t src_stride, const int* pairs_dev,
                         int npairs, const int64_t* segs_dev, int nseg, int64_t max_seg_bytes, hipStream_t st);

// engine: 0 = register-staged, 1 = LDS-staged (the Python default, kvx/agent.py COPY_ENGINE)
int llmd_kvx_copy_blocks2(void* dst, const void* src, int64_t dst_stride, int64_t src_stride, const int* pairs_dev,
                          int npairs, const int64_t* segs_dev, int nseg, int64_t max_seg_bytes, int engine,
                          hipStream_t st) {
  if (npairs == 0 || nseg == 0) return 0;
  if (engine == 0)
    return llmd_kvx_copy_blocks(dst, src, dst_stride, src_stride, pairs_dev, npairs, segs_dev, nseg, max_seg_bytes,
                                st);
  const int64_t nchunk = (max_seg_bytes + CP_CHUNK - 1) / CP_CHUNK;
  if (nchunk > 65535 || npairs > 65535 || nseg > 65535) return -2;
  dim3 grid((unsigned)nchunk, (unsigned)npairs, (unsigned)nseg);
  hipLaunchKernelGGL(copy_blocks_lds_kernel, grid, dim3(CP_NT), 0, st, (char*)dst, (const char*)src, dst_stride,
                     src_stride, pairs_dev, segs_dev);
  return (int)hipGetLastError();
}

int llmd_kvx_copy_blocks(void* dst, const void* src, int64_t dst_stride, int64_t src_stride,
                         const int* pairs_dev, int npairs, const int64_t* segs_dev, int nseg,
                         int64_t max_seg_bytes, hipStream_t st) {
  if (npairs == 0 || nseg == 0) return 0;
  const int64_t chunk = 256 * 1024;  // bytes per workgroup
  const int64_t nchunk = (max_seg_bytes + chunk - 1) / chunk;
  if (nchunk > 65535 || npairs > 65535 || nseg > 65535) return -2;
  dim3 grid((unsigned)nchunk, (unsigned)npairs, (unsigned)nseg);
  hipLaunchKernelGGL(copy_blocks_kernel, grid, dim3(NT), 0, st, (char*)dst, (const char*)src, dst_stride,
                     src_stride, pairs_dev, segs_dev, nseg, chunk);
  return (int)hipGetLastError();
}

// Export an IPC handle for the allocation containing `ptr`; returns the byte
// offset of ptr inside that allocation through *offset.
int llmd_kvx_ipc_export(const void* ptr, void* handle_out /*64 B*/, int64_t* offset) {
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr));
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, base);
  if (e != hipSuccess) return (int)e;
  std::memcpy(handle_out, &h, sizeof(h));
  *offset = (int64_t)((const char*)ptr - (const char*)base);
  return 0;
}

int llmd_kvx_ipc_open(const void* handle /*64 B*/, void** ptr_out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr_out, h, hipIpcMemLazyEnablePeerAccess);
}

int llmd_kvx_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

int llmd_kvx_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// DMA-engine path (SDMA over xGMI): one async copy per contiguous block range.
int llmd_kvx_dma_blocks(void* dst, const void* src, int64_t dst_stride, int64_t src_stride,
                        const int* pairs_host, int npairs, int64_t block_bytes, hipStream_t st) {
  for (int i = 0; i < npairs; ++i) {
    // coalesce runs of consecutive src and dst blocks into one copy
    int j = i;
    while (j + 1 < npairs && pairs_host[2 * (j + 1)] == pairs_host[2 * j] + 1 &&
           pairs_host[2 * (j + 1) + 1] == pairs_host[2 * j + 1] + 1 && dst_stride == block_bytes &&
           src_stride == block_bytes)
      ++j;
    const int n = j - i + 1;
    hipError_t e = hipMemcpyAsync((char*)dst + (int64_t)pairs_host[2 * i + 1] * dst_stride,
                                  (const char*)src + (int64_t)pairs_host[2 * i] * src_stride,
                                  (size_t)(n * block_bytes), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return (int)e;
    i = j;
  }
  return 0;
}
}
