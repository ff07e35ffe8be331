// kvx VMM pool: the producer's KV pool as ONE contiguous virtual range backed
// by several physical chunks (hipMemCreate, <= 2 GiB each), each exportable as
// a POSIX file descriptor (dmabuf). Measured on this image: importing a
// single >4 GiB allocation through hipIpcOpenMemHandle never returns, while
// chunks up to 4 GiB import instantly (scripts/ipc_probe.py), so a 100+ GB
// pool is exported chunk-wise. The importer maps the chunks back-to-back into
// its own reserved range, so the transfer kernels still see one base pointer
// and the attention kernels on the owner see a normal strided pool.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

extern "C" {

static hipMemAllocationProp vmm_prop(int device) {
  hipMemAllocationProp p = {};
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

int llmd_vmm_granularity(int device, size_t* gran) {
  hipMemAllocationProp p = vmm_prop(device);
  return (int)hipMemGetAllocationGranularity(gran, &p, hipMemAllocationGranularityRecommended);
}

static int map_access(void* base, size_t bytes, int device) {
  hipMemAccessDesc d = {};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = device;
  d.flags = hipMemAccessFlagsProtReadWrite;
  return (int)hipMemSetAccess(base, bytes, &d, 1);
}

// Allocate n_chunks * chunk_bytes as one virtual range; handles_out[n_chunks].
int llmd_vmm_alloc(int device, size_t chunk_bytes, int n_chunks, void** base_out, uint64_t* handles_out) {
  size_t total = chunk_bytes * (size_t)n_chunks;
  void* base = nullptr;
  hipError_t e = hipMemAddressReserve(&base, total, 0, nullptr, 0);
  if (e != hipSuccess) return (int)e;
  hipMemAllocationProp p = vmm_prop(device);
  for (int i = 0; i < n_chunks; ++i) {
    hipMemGenericAllocationHandle_t h;
    e = hipMemCreate(&h, chunk_bytes, &p, 0);
    if (e == hipSuccess) e = hipMemMap((char*)base + (size_t)i * chunk_bytes, chunk_bytes, 0, h, 0);
    if (e != hipSuccess) {
      for (int j = 0; j < i; ++j) {
        hipMemUnmap((char*)base + (size_t)j * chunk_bytes, chunk_bytes);
        hipMemRelease((hipMemGenericAllocationHandle_t)handles_out[j]);
      }
      hipMemAddressFree(base, total);
      return (int)e;
    }
    handles_out[i] = (uint64_t)h;
  }
  int rc = map_access(base, total, device);
  if (rc != 0) return rc;
  *base_out = base;
  return 0;
}

int llmd_vmm_export_fd(uint64_t handle, int* fd_out) {
  return (int)hipMemExportToShareableHandle((void*)fd_out, (hipMemGenericAllocationHandle_t)handle,
                                            hipMemHandleTypePosixFileDescriptor, 0);
}

// Import chunk fds (same chunk size) into one local virtual range mapped for `device`.
int llmd_vmm_import(const int* fds, int n_chunks, size_t chunk_bytes, int device, void** base_out,
                    uint64_t* handles_out) {
  size_t total = chunk_bytes * (size_t)n_chunks;
  void* base = nullptr;
  hipError_t e = hipMemAddressReserve(&base, total, 0, nullptr, 0);
  if (e != hipSuccess) return (int)e;
  for (int i = 0; i < n_chunks; ++i) {
    hipMemGenericAllocationHandle_t h;
    // HIP dereferences osHandle as an int* for POSIX fds (passing the fd value
    // itself, the CUDA convention, segfaults inside the runtime).
    int fd = fds[i];
    e = hipMemImportFromShareableHandle(&h, (void*)&fd, hipMemHandleTypePosixFileDescriptor);
    if (e == hipSuccess) e = hipMemMap((char*)base + (size_t)i * chunk_bytes, chunk_bytes, 0, h, 0);
    if (e != hipSuccess) return (int)e;
    handles_out[i] = (uint64_t)h;
  }
  int rc = map_access(base, total, device);
  if (rc != 0) return rc;
  *base_out = base;
  return 0;
}

int llmd_vmm_free(void* base, size_t chunk_bytes, int n_chunks, const uint64_t* handles) {
  int rc = 0;
  for (int i = 0; i < n_chunks; ++i) {
    hipError_t e = hipMemUnmap((char*)base + (size_t)i * chunk_bytes, chunk_bytes);
    if (e != hipSuccess) rc = (int)e;
    e = hipMemRelease((hipMemGenericAllocationHandle_t)handles[i]);
    if (e != hipSuccess) rc = (int)e;
  }
  hipError_t e = hipMemAddressFree(base, chunk_bytes * (size_t)n_chunks);
  return rc ? rc : (int)e;
}

}  // extern "C"
