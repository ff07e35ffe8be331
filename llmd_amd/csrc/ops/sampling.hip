// Token sampling over [B, V] logits.
//
// One workgroup per row, one pass over the row (16-byte loads):
//   * running max / sum-exp (online) -> log-softmax of the chosen token
//   * argmax of  logit/T + Gumbel(u)  with a counter-based RNG keyed by
//     (row seed, vocab index): an exact sample from softmax(logit/T)
//     (Gumbel-max), T <= 0 gives greedy argmax.
// Optional additive mask / penalties are applied by callers on the logits
// before this kernel. Top-k / top-p filtering is handled by `llmd_topk_topp_mask`.
#include "llmd_common.h"

using namespace llmd;

namespace {

constexpr int NT = 256;
constexpr float NEG_INF = -__builtin_huge_valf();

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// uniform in (0, 1)
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  const uint64_t h = mix64(seed ^ mix64(idx + 0x9e3779b97f4a7c15ull));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

struct Best {
  float v;
  int i;
};
__device__ __forceinline__ Best better(Best a, Best b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

// A row may be split over gridDim.y workgroups (batches smaller than the chip):
// each takes a contiguous range of 8-element chunks and writes its (max, sum-exp,
// best key, best index) to `part`; sample_merge_kernel folds them. The Gumbel
// keys depend only on (seed, vocab index), so the pick is the same for any split.
template <bool BF16>
__global__ __launch_bounds__(NT) void sample_kernel(const void* __restrict__ logits,
                                                    int64_t stride, int V,
                                                    const float* __restrict__ temps,
                                                    const int64_t* __restrict__ seeds,
                                                    int64_t* __restrict__ out_ids,
                                                    float* __restrict__ out_logprob, float* __restrict__ part) {
  const int row = blockIdx.x;
  const int nsp = gridDim.y, sp = blockIdx.y;
  const float T = temps ? temps[row] : 0.f;
  const bool greedy = !(T > 0.f);
  const float invT = greedy ? 1.f : 1.f / T;
  const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0ull;
  float mx = NEG_INF, se = 0.f;
  Best best{NEG_INF, 0x7fffffff};
  auto consume = [&](float x, int i) {
    // masked entries (-inf from top-k / top-p / min_p) add nothing; without the
    // guard a thread whose first entries are masked computes exp(-inf - -inf) = NaN
    if (x > mx) {
      se = se * __expf(mx - x) + 1.f;
      mx = x;
    } else if (x != NEG_INF) {
      se += __expf(x - mx);
    }
    float key = x;
    if (!greedy) {
      const float u = uniform01(seed, (uint64_t)i);
      key = x * invT - __logf(-__logf(u));
    }
    if (key > best.v || (key == best.v && i < best.i)) best = Best{key, i};
  };
  if (BF16) {
    const uint16_t* r = (const uint16_t*)logits + (int64_t)row * stride;
    const int nchunk = V / 8, per = (nchunk + nsp - 1) / nsp;
    const int c0 = sp * per, c1 = min(nchunk, c0 + per);
    for (int c = c0 + threadIdx.x; c < c1; c += NT) {
      float f[8];
      unpack8(*reinterpret_cast<const u32x4_t*>(r + c * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) consume(f[j], c * 8 + j);
    }
    if (sp == nsp - 1)
      for (int i = nchunk * 8 + threadIdx.x; i < V; i += NT) consume(bf2f(r[i]), i);
  } else {
    const float* r = (const float*)logits + (int64_t)row * stride;
    const int nchunk = V / 4, per = (nchunk + nsp - 1) / nsp;
    const int c0 = sp * per, c1 = min(nchunk, c0 + per);
    for (int c = c0 + threadIdx.x; c < c1; c += NT) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(r + c * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) consume(v[j], c * 4 + j);
    }
    if (sp == nsp - 1)
      for (int i = nchunk * 4 + threadIdx.x; i < V; i += NT) consume(r[i], i);
  }
  // wave reduce (max/sumexp and best)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float omx = __shfl_xor(mx, o, 64), ose = __shfl_xor(se, o, 64);
    const float nm = fmaxf(mx, omx);
    se = (mx == NEG_INF ? 0.f : se * __expf(mx - nm)) + (omx == NEG_INF ? 0.f : ose * __expf(omx - nm));
    mx = nm;
    Best ob{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, ob);
  }
  __shared__ float smx[NT / 64], sse[NT / 64], sbv[NT / 64];
  __shared__ int sbi[NT / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smx[w] = mx;
    sse[w] = se;
    sbv[w] = best.v;
    sbi[w] = best.i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = smx[0], S = sse[0];
    Best B{sbv[0], sbi[0]};
    for (int k = 1; k < NT / 64; ++k) {
      const float nm = fmaxf(M, smx[k]);
      S = (M == NEG_INF ? 0.f : S * __expf(M - nm)) + (smx[k] == NEG_INF ? 0.f : sse[k] * __expf(smx[k] - nm));
      M = nm;
      B = better(B, Best{sbv[k], sbi[k]});
    }
    if (nsp > 1) {
      float* pp = part + ((int64_t)row * nsp + sp) * 4;
      pp[0] = M;
      pp[1] = S;
      pp[2] = B.v;
      pp[3] = __int_as_float(B.i);
      return;
    }
    out_ids[row] = B.i;
    if (out_logprob) {
      const float xc = BF16 ? bf2f(((const uint16_t*)logits)[(int64_t)row * stride + B.i])
                            : ((const float*)logits)[(int64_t)row * stride + B.i];
      out_logprob[row] = xc - M - __logf(S);
    }
  }
}

template <bool BF16>
__global__ __launch_bounds__(64) void sample_merge_kernel(const void* __restrict__ logits, int64_t stride, int nsp,
                                                          const float* __restrict__ part, int64_t* __restrict__ out_ids,
                                                          float* __restrict__ out_logprob, int B) {
  const int row = blockIdx.x * 64 + threadIdx.x;
  if (row >= B) return;
  const float* pp = part + (int64_t)row * nsp * 4;
  float M = NEG_INF, S = 0.f;
  Best best{NEG_INF, 0x7fffffff};
  for (int k = 0; k < nsp; ++k) {
    const float mk = pp[4 * k], sk = pp[4 * k + 1];
    const float nm = fmaxf(M, mk);
    S = (M == NEG_INF ? 0.f : S * __expf(M - nm)) + (mk == NEG_INF ? 0.f : sk * __expf(mk - nm));
    M = nm;
    best = better(best, Best{pp[4 * k + 2], __float_as_int(pp[4 * k + 3])});
  }
  out_ids[row] = best.i;
  if (out_logprob) {
    const float xc = BF16 ? bf2f(((const uint16_t*)logits)[(int64_t)row * stride + best.i])
                          : ((const float*)logits)[(int64_t)row * stride + best.i];
    out_logprob[row] = xc - M - __logf(S);
  }
}

// Top-k / top-p (nucleus) filtering in place: entries outside the kept set are
// set to -inf. Threshold found by a 3-pass radix select on the order-preserving
// integer image of the (temperature-scaled) logits, with counts (top-k) and
// probability mass (top-p) histograms in LDS. One workgroup per row.
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int RBITS = 11, RBINS = 1 << RBITS;

__global__ __launch_bounds__(NT) void topk_topp_kernel(float* __restrict__ logits, int64_t stride,
                                                       int V, const int* __restrict__ topk,
                                                       const float* __restrict__ topp,
                                                       const float* __restrict__ temps) {
  const int row = blockIdx.x;
  float* r = logits + (int64_t)row * stride;
  const int k = topk ? topk[row] : 0;
  const float p = topp ? topp[row] : 1.f;
  const bool use_k = k > 0 && k < V;
  const bool use_p = p < 1.f;
  if (!use_k && !use_p) return;
  const float T = temps ? temps[row] : 1.f;
  const float invT = T > 0.f ? 1.f / T : 1.f;
  __shared__ uint32_t cnt[RBINS];
  __shared__ float mass[RBINS];
  __shared__ float red[NT / 64];
  __shared__ uint32_t s_prefix, s_need_cnt;
  __shared__ float s_need_mass;
  // max for stable exp
  float mx = NEG_INF;
  for (int i = threadIdx.x; i < V; i += NT) mx = fmaxf(mx, r[i]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float tot = 0.f;
  for (int i = threadIdx.x; i < V; i += NT) tot += __expf((r[i] - mx) * invT);
  tot = block_sum<NT>(tot, red);
  // find the threshold key: largest key K such that (count(key >= K) >= k) [top-k]
  // and (mass(key >= K) >= p*tot) [top-p]; keep every element with key >= K.
  uint32_t prefix = 0;
  uint32_t need_cnt = use_k ? (uint32_t)k : 0xffffffffu;
  float need_mass = use_p ? p * tot : 3.4e38f;
  const int shifts[3] = {21, 10, 0};
  const int widths[3] = {11, 11, 10};
  for (int pass = 0; pass < 3; ++pass) {
    const int sh = shifts[pass], wd = widths[pass];
    const uint32_t hi_mask = pass == 0 ? 0u : (0xffffffffu << (sh + wd));
    for (int b = threadIdx.x; b < RBINS; b += NT) {
      cnt[b] = 0;
      mass[b] = 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += NT) {
      const uint32_t key = fkey(r[i]);
      if ((key & hi_mask) == prefix) {
        const uint32_t bin = (key >> sh) & ((1u << wd) - 1);
        atomicAdd(&cnt[bin], 1u);
        atomicAdd(&mass[bin], __expf((r[i] - mx) * invT));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t c = 0;
      float ms = 0.f;
      int b = (1 << wd) - 1;
      for (; b > 0; --b) {
        const uint32_t nc = c + cnt[b];
        const float nm = ms + mass[b];
        if (nc >= need_cnt || nm >= need_mass) break;
        c = nc;
        ms = nm;
      }
      s_prefix = prefix | ((uint32_t)b << sh);
      s_need_cnt = need_cnt == 0xffffffffu ? need_cnt : need_cnt - c;
      s_need_mass = need_mass - ms;
    }
    __syncthreads();
    prefix = s_prefix;
    need_cnt = s_need_cnt;
    need_mass = s_need_mass;
    __syncthreads();
  }
  for (int i = threadIdx.x; i < V; i += NT)
    if (fkey(r[i]) < prefix) r[i] = NEG_INF;
}

}  // namespace

// rows split over nsp workgroups each (llmd_sample_splits), part: B * nsp * 4 floats
extern "C" int llmd_sample_splits(int B, int V) {
  if (B <= 0) return 1;
  int nsp = (512 + B - 1) / B;                      // ~2 workgroups per CU in total
  nsp = max(1, min(nsp, min(16, V / (8 * 2048))));  // keep >= 2k chunks of 8 per workgroup
  return nsp;
}

extern "C" void llmd_sample(const void* logits, int64_t stride, int B, int V, int is_bf16,
                            const float* temps, const int64_t* seeds, int64_t* out_ids,
                            float* out_logprob, float* part, int nsp, hipStream_t st) {
  if (B == 0) return;
  if (part == nullptr) nsp = 1;
  if (is_bf16)
    hipLaunchKernelGGL(sample_kernel<true>, dim3(B, nsp), dim3(NT), 0, st, logits, stride, V, temps,
                       seeds, out_ids, out_logprob, part);
  else
    hipLaunchKernelGGL(sample_kernel<false>, dim3(B, nsp), dim3(NT), 0, st, logits, stride, V, temps,
                       seeds, out_ids, out_logprob, part);
  if (nsp > 1) {
    if (is_bf16)
      hipLaunchKernelGGL(sample_merge_kernel<true>, dim3((B + 63) / 64), dim3(64), 0, st, logits, stride, nsp, part,
                         out_ids, out_logprob, B);
    else
      hipLaunchKernelGGL(sample_merge_kernel<false>, dim3((B + 63) / 64), dim3(64), 0, st, logits, stride, nsp, part,
                         out_ids, out_logprob, B);
  }
}

extern "C" void llmd_topk_topp_mask(float* logits, int64_t stride, int B, int V, const int* topk,
                                    const float* topp, const float* temps, hipStream_t st) {
  if (B == 0) return;
  hipLaunchKernelGGL(topk_topp_kernel, dim3(B), dim3(NT), 0, st, logits, stride, V, topk, topp,
                     temps);
}
