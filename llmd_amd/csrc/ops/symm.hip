// symm: an IPC symmetric heap over xGMI and the collectives built on it
// (SURVEY N05 NVSHMEM role, N08 DeepEP-LL role, K18 custom all-reduce).
//
// Every rank allocates one equal-size *uncached* device region
// (hipExtMallocWithFlags(hipDeviceMallocUncached)) and maps every peer's
// region through hipIpc. Uncached matters: peers write into our region over
// xGMI while our kernels run, and coarse-grained (L2-cached) memory would only
// be coherent at kernel boundaries. Layout of each region:
//
//   [0, SIG_BYTES)        signals: flag[ch][phase][block][src] (u32, written
//                         by peers), epoch[ch][block] (u32, local), err word
//   [SIG_BYTES, ...)      data: per-collective receive areas, double-buffered
//                         by epoch parity
//
// Synchronisation is per workgroup, no grid barrier: every collective runs a
// FIXED grid of G workgroups and uses the same element->workgroup partition on
// every rank, so workgroup b only waits for workgroup b of each peer. Each
// launch bumps a per-(channel, block) epoch kept in device memory, so a
// captured hipGraph replays correctly. Double-buffering by epoch parity makes
// an end barrier unnecessary: a peer can only overwrite the buffer we read at
// epoch e after passing barrier e+1, which needs our signal for e+1, which our
// stream only issues once our whole epoch-e kernel has completed.
//
// Pushing (remote stores) instead of pulling: each rank writes its data into
// peers' receive areas with 16-B stores, all 7 xGMI links in flight at once;
// the reduction then reads local HBM only.
//
// Every wait is bounded (LLMD_SYMM_TIMEOUT_S, default 20 s, on the 100 MHz
// s_memrealtime clock); on timeout the err word is set and the kernel
// finishes (with garbage) instead of hanging the GPU. symm_error() reports it,
// and the same timeout also sets a HOST-mapped word (fine-grained pinned host
// memory, llmd_symm_host_err) that the engine reads after every step with a
// plain load - no device sync - and turns into a fatal error before any token
// computed from a broken collective is emitted (parallel/symm.py check_health).
#include <cstdlib>
#include <cstring>

#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int MAXR = 8;          // ranks per heap (one node)
constexpr int G = 64;            // fixed workgroups per collective launch
constexpr int NT = 512;          // threads per workgroup
constexpr int NCH = 4;           // independent channels (streams / collectives)
constexpr int NPH = 2;           // barrier phases per launch
constexpr int64_t SIG_BYTES = 1 << 20;

struct Peers {
  char* base[MAXR];
  uint32_t* herr;        // host-mapped failure word (device address), or null
  uint64_t wait_ticks;   // barrier timeout in s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ uint32_t* flag_ptr(char* base, int ch, int ph, int b, int src) {
  return reinterpret_cast<uint32_t*>(base) + (((ch * NPH + ph) * G + b) * MAXR + src);
}
__device__ __forceinline__ uint32_t* epoch_ptr(char* base, int ch, int b) {
  return reinterpret_cast<uint32_t*>(base) + NCH * NPH * G * MAXR + ch * G + b;
}
__device__ __forceinline__ uint32_t* err_ptr(char* base) {
  return reinterpret_cast<uint32_t*>(base) + NCH * NPH * G * MAXR + NCH * G;
}

// Workgroup-entry: thread 0 bumps this block's epoch; everyone gets it via LDS.
__device__ __forceinline__ uint32_t next_epoch(char* self, int ch) {
  __shared__ uint32_t e_sh;
  if (threadIdx.x == 0) {
    uint32_t* ep = epoch_ptr(self, ch, blockIdx.x);
    uint32_t e = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(ep, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    e_sh = e;
  }
  __syncthreads();
  return e_sh;
}

// Combine runs under the epoch its dispatch opened (same parity buffers).
__device__ __forceinline__ uint32_t cur_epoch(char* self, int ch) {
  __shared__ uint32_t e_sh;
  if (threadIdx.x == 0) e_sh = __hip_atomic_load(epoch_ptr(self, ch, blockIdx.x), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return e_sh;
}

// Barrier among workgroup `blockIdx.x` of every rank: publish our data (every
// thread fences its own remote stores), signal each peer, wait for each peer.
__device__ __forceinline__ void block_barrier(const Peers& P, int nranks, int rank, int ch, int ph,
                                              uint32_t epoch) {
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < nranks && t != rank) {
    __hip_atomic_store(flag_ptr(P.base[t], ch, ph, blockIdx.x, rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (t < nranks && t != rank) {
    uint32_t* f = flag_ptr(P.base[rank], ch, ph, blockIdx.x, t);
    uint32_t* ew = err_ptr(P.base[rank]);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      uint32_t v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(v - epoch) >= 0) break;
      // A barrier of this rank already timed out (a dead peer): give up at
      // once, so only the first collective of a step or graph replay pays the
      // timeout and check_health fires after ~1x LLMD_SYMM_TIMEOUT_S, not Nx.
      if (__hip_atomic_load(ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > P.wait_ticks) {
        __hip_atomic_store(err_ptr(P.base[rank]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (P.herr != nullptr) __hip_atomic_store(P.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__device__ __forceinline__ void acc8(float* a, const u32x4_t v) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] += f[i];
}

// ------------------------------------------------------------ all-reduce
// One-shot: packet q (16 B) of the input is handled by workgroup q % G on every
// rank. Push q to every peer's area[par][rank][q], barrier, sum the N copies.
__global__ __launch_bounds__(NT) void ar_oneshot_kernel(Peers P, int nranks, int rank, int ch,
                                                        int64_t data_off, int64_t slot_bytes,
                                                        const u32x4_t* __restrict__ in,
                                                        u32x4_t* __restrict__ out, int64_t npk) {
  const uint32_t epoch = next_epoch(P.base[rank], ch);
  const int par = epoch & 1;
  const int64_t area = data_off + (int64_t)par * nranks * slot_bytes;
  for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q < npk; q += (int64_t)G * NT) {
    const u32x4_t v = in[q];
    for (int p = 0; p < nranks; ++p) {
      if (p == rank) continue;
      u32x4_t* dst = reinterpret_cast<u32x4_t*>(P.base[p] + area + (int64_t)rank * slot_bytes);
      dst[q] = v;
    }
  }
  block_barrier(P, nranks, rank, ch, 0, epoch);
  for (int64_t q = (int64_t)blockIdx.x * NT + threadIdx.x; q < npk; q += (int64_t)G * NT) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < nranks; ++p) {
      const u32x4_t* src = p == rank ? in : reinterpret_cast<const u32x4_t*>(
                                                P.base[rank] + area + (int64_t)p * slot_bytes);
      acc8(a, src[q]);
    }
    out[q] = pack8(a);
  }
}

// Two-shot: reduce-scatter then all-gather. The packets split into nranks
// contiguous slices of `spk` packets (last one may be short); packet j of a
// slice belongs to workgroup j % G on every rank.
__global__ __launch_bounds__(NT) void ar_twoshot_kernel(Peers P, int nranks, int rank, int ch,
                                                        int64_t data_off, int64_t slot_bytes,
                                                        const u32x4_t* __restrict__ in,
                                                        u32x4_t* __restrict__ out, int64_t npk,
                                                        int64_t spk) {
  const uint32_t epoch = next_epoch(P.base[rank], ch);
  const int par = epoch & 1;
  // area1[par][src][spk] receives slices to reduce; area2[par][src][spk] receives reduced slices
  const int64_t a1 = data_off + (int64_t)par * 2 * nranks * slot_bytes;
  const int64_t a2 = a1 + (int64_t)nranks * slot_bytes;
  for (int o = 0; o < nranks; ++o) {
    if (o == rank) continue;
    const int64_t s0 = (int64_t)o * spk;
    const int64_t n = min(spk, npk - s0);
    u32x4_t* dst = reinterpret_cast<u32x4_t*>(P.base[o] + a1 + (int64_t)rank * slot_bytes);
    for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (int64_t)G * NT) dst[j] = in[s0 + j];
  }
  block_barrier(P, nranks, rank, ch, 0, epoch);
  {
    const int64_t s0 = (int64_t)rank * spk;
    const int64_t n = max((int64_t)0, min(spk, npk - s0));
    for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (int64_t)G * NT) {
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < nranks; ++p) {
        const u32x4_t v = p == rank ? in[s0 + j]
                                    : reinterpret_cast<const u32x4_t*>(P.base[rank] + a1 +
                                                                       (int64_t)p * slot_bytes)[j];
        acc8(a, v);
      }
      const u32x4_t r = pack8(a);
      out[s0 + j] = r;
      for (int p = 0; p < nranks; ++p) {
        if (p == rank) continue;
        reinterpret_cast<u32x4_t*>(P.base[p] + a2 + (int64_t)rank * slot_bytes)[j] = r;
      }
    }
  }
  block_barrier(P, nranks, rank, ch, 1, epoch);
  for (int o = 0; o < nranks; ++o) {
    if (o == rank) continue;
    const int64_t s0 = (int64_t)o * spk;
    const int64_t n = min(spk, npk - s0);
    const u32x4_t* src = reinterpret_cast<const u32x4_t*>(P.base[rank] + a2 + (int64_t)o * slot_bytes);
    for (int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x; j < n; j += (int64_t)G * NT) out[s0 + j] = src[j];
  }
}

// ------------------------------------------------------------ EP dispatch / combine
// Fixed-shape (LL) exchange for wide-EP decode: every rank contributes exactly
// R token rows (its T real tokens + padding). Receive area on each rank:
//   rx[par][src][R][d] bf16, rid[par][src][R][k] i32 (local expert | -1),
//   rw[par][src][R][k] f32
// Token t of rank r is written to rank p only if one of its top-k experts lives
// on p; otherwise only its id row (all -1) is written, so p's grouped GEMM
// skips it. Rows t are owned by workgroup t % G (same on every rank).
struct EpLayout {
  int64_t rx, rid, rw, cb;  // byte offsets of the four areas (parity 0)
  int64_t par_stride;       // bytes between parity 0 and 1
  int64_t rxq, rxs;         // fp8 dispatch: e4m3 rows [src][R][dp] + group scales [src][R][dp/128] (or -1)
};

__global__ __launch_bounds__(NT) void ep_dispatch_kernel(Peers P, int nranks, int rank, int ch, EpLayout L,
                                                         const uint16_t* __restrict__ x, int64_t xs,
                                                         const int* __restrict__ ids, const float* __restrict__ w,
                                                         int T, int R, int d, int k, int E_local) {
  const uint32_t epoch = next_epoch(P.base[rank], ch);
  const int64_t po = (int64_t)(epoch & 1) * L.par_stride;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  constexpr int NW = NT / 64;
  // one wave per (token, dest rank); t % G == blockIdx.x
  for (int64_t i = wv;; i += NW) {
    const int64_t t = blockIdx.x + (int64_t)G * (i / nranks);
    const int p = (int)(i % nranks);
    if (t >= R) break;
    char* pb = P.base[p];
    int* rid = reinterpret_cast<int*>(pb + L.rid + po) + ((int64_t)rank * R + t) * k;
    float* rw = reinterpret_cast<float*>(pb + L.rw + po) + ((int64_t)rank * R + t) * k;
    bool any = false;
    int lid = -1;
    float lw = 0.f;
    if (t < T && ln < k) {
      const int e = ids[t * k + ln];
      if (e >= p * E_local && e < (p + 1) * E_local) {
        lid = e - p * E_local;
        lw = w[t * k + ln];
      }
    }
    any = __any(lid >= 0);
    if (ln < k) {
      rid[ln] = lid;
      rw[ln] = lw;
    }
    if (any) {
      const u32x4_t* src = reinterpret_cast<const u32x4_t*>(x + t * xs);
      u32x4_t* dst = reinterpret_cast<u32x4_t*>(pb + L.rx + po) + ((int64_t)rank * R + t) * (d / 8);
      for (int c = ln; c < d / 8; c += 64) dst[c] = src[c];
    }
  }
  block_barrier(P, nranks, rank, ch, 0, epoch);
}

// FP8 dispatch (DeepEP-LL with fp8 fused in): the same exchange, but a token
// row travels as e4m3fn with one power-of-two (E8M0-exact) scale per 128
// columns - quantised in registers by the sending wave, the same numerics as
// ops.quant_fp8_groups - into rxq [src][R][dp] / rxs [src][R][dp / 128]
// (dp = d rounded up to 128, zero padded): half the xGMI bytes of bf16, and the
// block-fp8 grouped GEMM consumes the rows without a quantisation pass.
__global__ __launch_bounds__(NT) void ep_dispatch_fp8_kernel(Peers P, int nranks, int rank, int ch, EpLayout L,
                                                             const uint16_t* __restrict__ x, int64_t xs,
                                                             const int* __restrict__ ids,
                                                             const float* __restrict__ w, int T, int R, int d,
                                                             int k, int E_local) {
  const uint32_t epoch = next_epoch(P.base[rank], ch);
  const int64_t po = (int64_t)(epoch & 1) * L.par_stride;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  constexpr int NW = NT / 64;
  const int ng = (d + 127) / 128, dp = ng * 128;
  for (int64_t i = wv;; i += NW) {
    const int64_t t = blockIdx.x + (int64_t)G * (i / nranks);
    const int p = (int)(i % nranks);
    if (t >= R) break;
    char* pb = P.base[p];
    const int64_t row = (int64_t)rank * R + t;
    int* rid = reinterpret_cast<int*>(pb + L.rid + po) + row * k;
    float* rw = reinterpret_cast<float*>(pb + L.rw + po) + row * k;
    int lid = -1;
    float lw = 0.f;
    if (t < T && ln < k) {
      const int e = ids[t * k + ln];
      if (e >= p * E_local && e < (p + 1) * E_local) {
        lid = e - p * E_local;
        lw = w[t * k + ln];
      }
    }
    const bool any = __any(lid >= 0);
    if (ln < k) {
      rid[ln] = lid;
      rw[ln] = lw;
    }
    if (!any) continue;
    const uint16_t* src = x + t * xs;
    uint8_t* dq = reinterpret_cast<uint8_t*>(pb + L.rxq + po) + row * dp;
    float* ds = reinterpret_cast<float*>(pb + L.rxs + po) + row * ng;
    // 16 lanes x 8 columns per 128-column group, 4 groups per wave pass
    for (int g0 = 0; g0 < ng; g0 += 4) {
      const int g = g0 + (ln >> 4), c = g * 128 + (ln & 15) * 8;
      float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (g < ng && c < d) unpack8(*reinterpret_cast<const u32x4_t*>(src + c), f);
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) a = fmaxf(a, fabsf(f[j]));
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
      const float s = pow2_ceil(fmaxf(a / FP8_MAX, 1e-12f));
      const float inv = 1.f / s;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= inv;
      if (g < ng) {
        *reinterpret_cast<u32x2_t*>(dq + c) = f32x8_to_fp8(f);
        if ((ln & 15) == 0) ds[g] = s;
      }
    }
  }
  block_barrier(P, nranks, rank, ch, 0, epoch);
}

// y rows [src][R][d] (bf16, weighted partial sums of our local experts) go back
// to their owners' combine area cb[par][from][R][d]; the owner sums the copies
// of ranks that hold one of the token's experts.
__global__ __launch_bounds__(NT) void ep_combine_kernel(Peers P, int nranks, int rank, int ch, EpLayout L,
                                                        const uint16_t* __restrict__ y, int64_t ys,
                                                        const int* __restrict__ ids, int T, int R, int d, int k,
                                                        int E_local, uint16_t* __restrict__ out, int64_t os) {
  const uint32_t epoch = cur_epoch(P.base[rank], ch);  // the epoch of the matching dispatch
  const int64_t po = (int64_t)(epoch & 1) * L.par_stride;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  constexpr int NW = NT / 64;
  const int* my_rid = reinterpret_cast<const int*>(P.base[rank] + L.rid + po);
  // send: row (s, t) for t % G == blockIdx.x; one wave per row
  for (int64_t i = wv; ; i += NW) {
    const int64_t t = blockIdx.x + (int64_t)G * (i / nranks);
    const int s = (int)(i % nranks);
    if (t >= R) break;
    const int* r = my_rid + ((int64_t)s * R + t) * k;
    const bool valid = __any(ln < k && r[ln] >= 0);
    if (!valid) continue;
    const u32x4_t* src = reinterpret_cast<const u32x4_t*>(y + ((int64_t)s * R + t) * ys);
    u32x4_t* dst = reinterpret_cast<u32x4_t*>(P.base[s] + L.cb + po) + ((int64_t)rank * R + t) * (d / 8);
    for (int c = ln; c < d / 8; c += 64) dst[c] = src[c];
  }
  block_barrier(P, nranks, rank, ch, 1, epoch);
  // receive: token t sums the copies from ranks holding one of its experts
  const u32x4_t* cb = reinterpret_cast<const u32x4_t*>(P.base[rank] + L.cb + po);
  for (int64_t i = wv;; i += NW) {
    const int64_t t = blockIdx.x + (int64_t)G * i;
    if (t >= T) break;
    uint32_t mask = 0;
    if (ln < k) {
      const int e = ids[t * k + ln];
      if (e >= 0) mask = 1u << (e / E_local);
    }
    // OR-reduce the rank mask over the wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mask |= __shfl_xor(mask, o, 64);
    for (int c = ln; c < d / 8; c += 64) {
      float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < nranks; ++p)
        if (mask & (1u << p)) acc8(a, cb[((int64_t)p * R + t) * (d / 8) + c]);
      reinterpret_cast<u32x4_t*>(out + t * os)[c] = pack8(a);
    }
  }
}

}  // namespace

extern "C" {

int llmd_symm_alloc(size_t bytes, void** out) {
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, SIG_BYTES);
  if (e != hipSuccess) return (int)e;
  e = hipDeviceSynchronize();
  *out = p;
  return (int)e;
}

int llmd_symm_free(void* p) { return (int)hipFree(p); }

int64_t llmd_symm_sig_bytes() { return SIG_BYTES; }
int llmd_symm_grid() { return G; }
int llmd_symm_max_ranks() { return MAXR; }
int llmd_symm_channels() { return NCH; }

int llmd_symm_error(const void* self, uint32_t* err) {
  const char* b = (const char*)self;
  return (int)hipMemcpy(err, b + (NCH * NPH * G * MAXR + NCH * G) * 4, 4, hipMemcpyDeviceToHost);
}

int llmd_symm_clear_error(void* self) {
  return (int)hipMemset((char*)self + (NCH * NPH * G * MAXR + NCH * G) * 4, 0, 4);
}

// One fine-grained (coherent) mapped host word per process: every symm launch
// carries its device address, so it must exist before any graph is captured
// (SymmHeap creates it).
static uint32_t* g_herr_host = nullptr;
static uint32_t* g_herr_dev = nullptr;

int llmd_symm_host_err(int64_t* host_ptr) {
  if (g_herr_host == nullptr) {
    void* h = nullptr;
    hipError_t e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return (int)e;
    std::memset(h, 0, 64);
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) return (int)e;
    g_herr_host = (uint32_t*)h;
    g_herr_dev = (uint32_t*)d;
  }
  *host_ptr = (int64_t)(uintptr_t)g_herr_host;
  return 0;
}

// Barrier timeout: LLMD_SYMM_TIMEOUT_S (default 20 s, the order of the reference's
// NCCL heartbeat timeout of 15 s) - long enough for any lock-step skew between
// ranks (a long prefill chunk on one DP rank), short enough to fail a wedged
// replica quickly.
static uint64_t wait_ticks() {
  static uint64_t t = 0;
  if (t == 0) {
    const char* e = std::getenv("LLMD_SYMM_TIMEOUT_S");
    double sec = e != nullptr ? std::atof(e) : 20.0;
    if (!(sec > 0.0)) sec = 20.0;
    t = (uint64_t)(sec * 1e8);  // s_memrealtime runs at 100 MHz
  }
  return t;
}

static Peers make_peers(const int64_t* bases, int n) {
  Peers P = {};
  for (int i = 0; i < n; ++i) P.base[i] = (char*)bases[i];
  P.herr = g_herr_dev;
  P.wait_ticks = wait_ticks();
  return P;
}

// mode 1 = one-shot, 2 = two-shot; npk = bytes / 16
int llmd_symm_all_reduce(const int64_t* bases, int nranks, int rank, int ch, int mode, int64_t data_off,
                         int64_t slot_bytes, const void* in, void* out, int64_t npk, hipStream_t st) {
  if (nranks < 2 || nranks > MAXR || ch < 0 || ch >= NCH) return -1;
  Peers P = make_peers(bases, nranks);
  if (mode == 1) {
    if (npk * 16 > slot_bytes) return -2;
    hipLaunchKernelGGL(ar_oneshot_kernel, dim3(G), dim3(NT), 0, st, P, nranks, rank, ch, data_off, slot_bytes,
                       (const u32x4_t*)in, (u32x4_t*)out, npk);
  } else {
    const int64_t spk = (npk + nranks - 1) / nranks;
    if (spk * 16 > slot_bytes) return -2;
    hipLaunchKernelGGL(ar_twoshot_kernel, dim3(G), dim3(NT), 0, st, P, nranks, rank, ch, data_off, slot_bytes,
                       (const u32x4_t*)in, (u32x4_t*)out, npk, spk);
  }
  return (int)hipGetLastError();
}

int llmd_symm_ep_dispatch(const int64_t* bases, int nranks, int rank, int ch, const int64_t* lay,
                          const void* x, int64_t xs, const int* ids, const float* w, int T, int R, int d, int k,
                          int E_local, int fp8, hipStream_t st) {
  if (nranks < 1 || nranks > MAXR || k > 64 || d % 8) return -1;
  EpLayout L{lay[0], lay[1], lay[2], lay[3], lay[4], lay[5], lay[6]};
  if (fp8) {
    if (L.rxq < 0 || L.rxs < 0) return -3;
    hipLaunchKernelGGL(ep_dispatch_fp8_kernel, dim3(G), dim3(NT), 0, st, make_peers(bases, nranks), nranks, rank,
                       ch, L, (const uint16_t*)x, xs, ids, w, T, R, d, k, E_local);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(ep_dispatch_kernel, dim3(G), dim3(NT), 0, st, make_peers(bases, nranks), nranks, rank, ch, L,
                     (const uint16_t*)x, xs, ids, w, T, R, d, k, E_local);
  return (int)hipGetLastError();
}

int llmd_symm_ep_combine(const int64_t* bases, int nranks, int rank, int ch, const int64_t* lay, const void* y,
                         int64_t ys, const int* ids, int T, int R, int d, int k, int E_local, void* out, int64_t os,
                         hipStream_t st) {
  if (nranks < 1 || nranks > MAXR || k > 64 || d % 8) return -1;
  EpLayout L{lay[0], lay[1], lay[2], lay[3], lay[4], lay[5], lay[6]};
  hipLaunchKernelGGL(ep_combine_kernel, dim3(G), dim3(NT), 0, st, make_peers(bases, nranks), nranks, rank, ch, L,
                     (const uint16_t*)y, ys, ids, T, R, d, k, E_local, (uint16_t*)out, os);
  return (int)hipGetLastError();
}

}  // extern "C"
