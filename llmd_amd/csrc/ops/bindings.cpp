// Python bindings for the llmd_amd HIP op library. Host C++ only (compiled by
// g++ against the torch headers); the kernels live in the *.hip translation
// units and are reached through their extern "C" launchers. Every binding
// checks device, dtype, contiguity of the inner dimension and the shapes the
// kernel's grid assumes, so a bad call raises instead of faulting the GPU.
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <pybind11/stl.h>

#include <map>
#include <mutex>
#include <memory>
#include <vector>

extern "C" {
void llmd_rms_norm(void*, int64_t, const void*, int64_t, const void*, int, int, float, hipStream_t);
void llmd_layer_norm(void*, int64_t, void*, int64_t, void*, int64_t, const void*, const void*, int, int, float,
                     hipStream_t);
void llmd_fused_add_rms_norm(void*, int64_t, void*, int64_t, const void*, int, int, float,
                             hipStream_t);
int llmd_qk_rms_norm(void*, int64_t, const void*, const void*, int, int, int, int, float, hipStream_t);
void llmd_rope_cache(void*, int64_t, const int64_t*, const float*, int, int, int, int,
                     const int64_t*, void*, void*, int64_t, int, int, int, int, float, float, hipStream_t);
void llmd_gated_act(void*, int64_t, const void*, int64_t, int, int, int, float, float, hipStream_t);
int llmd_paged_decode(const void*, int64_t, const void*, const void*, int64_t, int, const int*, int,
                      const int*, int, int, int, int, float, int, const float*, int, int, void*,
                      int64_t, float*, float*, int, float, float, const int*, const int*, const int*,
                      const int*, int, int, int, const int*, hipStream_t);
int llmd_paged_prefill(const void*, int64_t, const void*, const void*, int64_t, int, const int*, int,
                       const int*, const int*, const int*, const int*, int, int, int, int, float,
                       int, const float*, void*, int64_t, int, float, float, hipStream_t);
int llmd_prefill_tokens_per_item(int, int, int, int, int);
void llmd_sample(const void*, int64_t, int, int, int, const float*, const int64_t*, int64_t*, float*,
                 float*, int, hipStream_t);
int llmd_sample_splits(int, int);
void llmd_topk_topp_mask(float*, int64_t, int, int, const int*, const float*, const float*,
                         hipStream_t);
int llmd_kvx_copy_blocks(void*, const void*, int64_t, int64_t, const int*, int, const int64_t*, int,
                         int64_t, hipStream_t);
int llmd_kvx_copy_blocks2(void*, const void*, int64_t, int64_t, const int*, int, const int64_t*, int, int64_t, int,
                          hipStream_t);
int llmd_kvx_ipc_export(const void*, void*, int64_t*);
int llmd_kvx_ipc_open(const void*, void**);
int llmd_kvx_ipc_close(void*);
int llmd_mla_attention(const void*, int64_t, const void*, int64_t, int, const int*, int, const int*,
                       const int*, int, int, float, int, int, void*, int64_t, float*, float*, int, float,
                       const int*, hipStream_t);
int llmd_mla_rope_cache(const void*, int64_t, void*, int64_t, const void*, int64_t, const void*, int64_t,
                        const int64_t*, const float*, int, int, const int64_t*, void*, int64_t, int, int, float,
                        hipStream_t);
int llmd_lora_bgmv(const void*, int64_t, const void*, const void*, int, int, int, int, const int*, float*, void*,
                   int64_t, hipStream_t);
int llmd_skinny_gemm(const void*, int64_t, const void*, int64_t, int, int, int, int, int, int, void*, int64_t,
                     float*, hipStream_t);
int llmd_dgemm_supported(int, int, int);
int llmd_mgemm(const void*, int64_t, const void*, int64_t, int, int, int, int, int, int, void*, int64_t, float*,
               int*, hipStream_t);
int llmd_mgemm_lds(int, int, int);
int llmd_mgemm_partials(const void*, int64_t, const void*, int64_t, int, int, int, int, int, int, float*, hipStream_t);
int llmd_reduce_rope_cache(const float*, int, int, void*, int64_t, const int64_t*, const float*, int, int, int, int,
                           const int64_t*, void*, void*, int64_t, int, int, int, int, float, float, hipStream_t);
int llmd_mgemm_add_rmsnorm(const void*, int64_t, const void*, int64_t, int, int, int, int, int, int, float*, void*,
                           int64_t, const void*, float, void*, int64_t, hipStream_t);
int llmd_mgemm_silu(const void*, int64_t, const void*, int64_t, int, int, int, int, int, void*, int64_t, hipStream_t);
int llmd_pgemm(const void*, int64_t, const void*, int64_t, void*, int64_t, int, int, int, int, int, void*,
               hipStream_t);
int64_t llmd_pgemm_ws_bytes(int, int, int, int, int);
int llmd_pgemm_fp8(const void*, int64_t, const float*, const void*, int64_t, const float*, void*, int64_t, int, int,
                   int, int, void*, int, hipStream_t);
int64_t llmd_pgemm_fp8_ws_bytes(int, int, int, int);
int llmd_mgemm_fp8(const void*, int64_t, const float*, const void*, int64_t, const float*, int, int, int, int, int,
                   int, void*, int64_t, float*, int*, hipStream_t);
int llmd_vmm_granularity(int, size_t*);
int llmd_vmm_alloc(int, size_t, int, void**, uint64_t*);
int llmd_vmm_export_fd(uint64_t, int*);
int llmd_vmm_import(const int*, int, size_t, int, void**, uint64_t*);
int llmd_vmm_free(void*, size_t, int, const uint64_t*);
int llmd_kvx_handle_size();
int llmd_kvx_dma_blocks(void*, const void*, int64_t, int64_t, const int*, int, int64_t, hipStream_t);
void llmd_moe_topk(const float*, int, int, int, int, const float*, int, int, int, float, int*, float*,
                   hipStream_t);
void llmd_moe_align(const int*, int, int, int, int*, int*, int*, int, int*, int*, hipStream_t);
int llmd_moe_gemm_tile_m();
void llmd_moe_gemm(const void*, int64_t, int, const int*, const int*, int, const void*, int64_t, int, int,
                   void*, int64_t, int, int, float, float, int, const void*, hipStream_t);
void llmd_moe_combine(const void*, int64_t, const int*, const float*, int, int, int, void*, int64_t,
                      hipStream_t);
int llmd_quant_fp8_rows(const void*, int64_t, void*, int64_t, float*, int, int, hipStream_t);
void llmd_rms_norm_quant(void*, int64_t, float*, const void*, int64_t, void*, int64_t, const void*, int, int, float,
                         hipStream_t);
void llmd_gated_act_quant(void*, int64_t, float*, const void*, int64_t, int, int, int, float, float, hipStream_t);
int llmd_quant_fp8_groups(const void*, int64_t, void*, int64_t, float*, int64_t, int, int, hipStream_t);
int llmd_quant_fp8_groups_padded(const void*, int64_t, void*, int64_t, float*, int64_t, int, int, int, const int*,
                                 hipStream_t);
void llmd_moe_gemm_fp8(const void*, int64_t, const float*, int64_t, int, const int*, const int*, int, const void*,
                       int64_t, const float*, int, int, void*, int64_t, int, int, float, float, int, const void*,
                       hipStream_t);
int llmd_moe_gemm3_fp8(const void*, int64_t, const float*, int64_t, int, const int*, const int*, int, const void*,
                       int64_t, const float*, int, int, void*, int64_t, int, int, float, float, int, const void*,
                       void*, int64_t, float*, int64_t, hipStream_t);
int llmd_moe_gemm3_tile_m();
int llmd_moe_gemm4_bf16(const void*, int64_t, int, const int*, const int*, int, const void*, int64_t, int, int, void*,
                        int64_t, int, int, float, float, int, const void*, int64_t, int, hipStream_t);
int llmd_moe_gemm8_bf16(const void*, int64_t, int, const int*, const int*, const int*, int, const void*, int64_t, int,
                        int, void*, int64_t, int, int, float, float, int, const void*, int64_t, int, hipStream_t);
int llmd_moe_gemm4_fp8(const void*, int64_t, const float*, int64_t, int, const int*, const int*, int, const void*,
                       int64_t, const float*, int, int, void*, int64_t, int, int, float, float, int, const void*,
                       int64_t, int, hipStream_t);
int llmd_moe_gemm8_fp8(const void*, int64_t, const float*, int64_t, int, const int*, const int*, const int*, int,
                       const void*, int64_t, const float*, int, int, void*, int64_t, int, int, float, float, int,
                       const void*, int64_t, int, hipStream_t);
int llmd_moe_gemm3_bf16(const void*, int64_t, int, const int*, const int*, int, const void*, int64_t, int, int, void*,
                        int64_t, int, int, float, float, int, const void*, hipStream_t);
int llmd_symm_alloc(size_t, void**);
int llmd_symm_free(void*);
int64_t llmd_symm_sig_bytes();
int llmd_symm_grid();
int llmd_symm_max_ranks();
int llmd_symm_channels();
int llmd_symm_error(const void*, uint32_t*);
int llmd_symm_clear_error(void*);
int llmd_symm_host_err(int64_t*);
int llmd_symm_all_reduce(const int64_t*, int, int, int, int, int64_t, int64_t, const void*, void*, int64_t,
                         hipStream_t);
int llmd_symm_ep_dispatch(const int64_t*, int, int, int, const int64_t*, const void*, int64_t, const int*,
                          const float*, int, int, int, int, int, int, hipStream_t);
int llmd_symm_ep_combine(const int64_t*, int, int, int, const int64_t*, const void*, int64_t, const int*, int, int,
                         int, int, int, void*, int64_t, hipStream_t);
}

namespace {

// Kernels launch on the tensor's device even from threads whose current device
// differs (engine / kvx threads); CPU tensors fall through to the CHECKs.
std::optional<c10::DeviceIndex> dev_of(const torch::Tensor& t) {
  if (t.is_cuda()) return t.get_device();
  return std::nullopt;
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_INNER(x) TORCH_CHECK((x).stride(-1) == 1, #x " inner dim must be contiguous")
#define CHECK_DT(x, t) TORCH_CHECK((x).scalar_type() == (t), #x " has wrong dtype")

void rms_norm(torch::Tensor out, torch::Tensor x, torch::Tensor w, double eps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(out));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_BF16(w);
  CHECK_INNER(x); CHECK_INNER(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && w.is_contiguous(), "rms_norm: 2-D x/out");
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && w.numel() == d && out.size(1) == d && out.size(0) == x.size(0),
              "rms_norm shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "rms_norm: 16-B aligned rows");
  llmd_rms_norm(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), x.size(0), d,
                (float)eps, cur_stream());
}

void qk_rms_norm(torch::Tensor qkv, torch::Tensor qw, torch::Tensor kw, int64_t Hq, int64_t Hkv, double eps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(qkv));
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_BF16(qw); CHECK_BF16(kw);
  CHECK_INNER(qkv);
  TORCH_CHECK(qkv.dim() == 2, "qk_rms_norm: qkv [T, (Hq+2Hkv)*D]");
  const int64_t D = qw.numel();
  TORCH_CHECK(kw.numel() == D && qw.is_contiguous() && kw.is_contiguous(), "qk_rms_norm: weights [D]");
  TORCH_CHECK(D == 64 || D == 128 || D == 256, "qk_rms_norm: head dim 64 / 128 / 256");
  TORCH_CHECK(qkv.size(1) >= (Hq + Hkv) * D, "qk_rms_norm: qkv narrower than (Hq + Hkv) * D");
  const int rc = llmd_qk_rms_norm(qkv.data_ptr(), qkv.stride(0), qw.data_ptr(), kw.data_ptr(), qkv.size(0),
                                  (int)Hq, (int)Hkv, (int)D, (float)eps, cur_stream());
  TORCH_CHECK(rc == 0, "qk_rms_norm: unsupported head dim");
}

void fused_add_rms_norm(torch::Tensor x, torch::Tensor residual, torch::Tensor w, double eps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_BF16(w);
  CHECK_INNER(x); CHECK_INNER(residual);
  TORCH_CHECK(x.dim() == 2 && residual.sizes() == x.sizes(), "fused_add_rms_norm shape");
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && w.numel() == d && w.is_contiguous(), "fused_add_rms_norm d");
  TORCH_CHECK(x.stride(0) % 8 == 0 && residual.stride(0) % 8 == 0, "16-B aligned rows");
  llmd_fused_add_rms_norm(x.data_ptr(), x.stride(0), residual.data_ptr(), residual.stride(0),
                          w.data_ptr(), x.size(0), d, (float)eps, cur_stream());
}

// out = layernorm(x) w + b, or (residual given) residual += x; x = layernorm(residual) w + b in place
void layer_norm(torch::Tensor out, torch::Tensor x, c10::optional<torch::Tensor> residual, torch::Tensor w,
                torch::Tensor b, double eps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_BF16(w); CHECK_BF16(b);
  CHECK_INNER(x); CHECK_INNER(out);
  TORCH_CHECK(x.dim() == 2 && out.sizes() == x.sizes(), "layer_norm: 2-D x/out of one shape");
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && w.numel() == d && b.numel() == d && w.is_contiguous() && b.is_contiguous(),
              "layer_norm: d % 8 == 0, contiguous w/b of d elements");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "layer_norm: 16-B aligned rows");
  void* rp = nullptr;
  int64_t rs = 0;
  if (residual.has_value()) {
    CHECK_BF16(*residual); CHECK_INNER(*residual);
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->stride(0) % 8 == 0, "layer_norm residual shape");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  llmd_layer_norm(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), rp, rs, w.data_ptr(), b.data_ptr(),
                  x.size(0), d, (float)eps, cur_stream());
}

// KV caches are bf16 or fp8 e4m3fn (OCP, gfx950's native fp8)
bool is_fp8_cache(const torch::Tensor& c) {
  TORCH_CHECK(c.is_cuda(), "cache must be a GPU tensor");
  const auto t = c.scalar_type();
  TORCH_CHECK(t == at::kBFloat16 || t == at::kFloat8_e4m3fn, "KV cache must be bf16 or float8_e4m3fn");
  return t == at::kFloat8_e4m3fn;
}

// qkv [T, (Hq+2Hkv)*D]; k_cache/v_cache: per-layer strided views
// [num_blocks, Hkv, bs, D] (block stride arbitrary, inner [Hkv,bs,D] contiguous)
void rope_cache(torch::Tensor qkv, torch::Tensor positions, torch::Tensor cos_sin, int64_t Hq,
                int64_t Hkv, int64_t D, torch::Tensor slots, torch::Tensor k_cache,
                torch::Tensor v_cache, bool neox, double k_scale, double v_scale) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(qkv));
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_INNER(qkv);
  CHECK_DT(positions, at::kLong); CHECK_DT(slots, at::kLong); CHECK_DT(cos_sin, at::kFloat);
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) >= (Hq + 2 * Hkv) * D, "rope_cache: qkv width");
  const int T = qkv.size(0);
  TORCH_CHECK(positions.numel() == T && slots.numel() == T, "rope_cache: T mismatch");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.is_contiguous(), "cos_sin 2-D contiguous");
  const int rot = cos_sin.size(1);
  TORCH_CHECK(rot % 16 == 0 && rot <= D && D % 8 == 0, "rope_cache: rotary dim");
  TORCH_CHECK(qkv.stride(0) % 8 == 0, "rope_cache: 16-B aligned rows");
  const bool f8 = is_fp8_cache(k_cache);
  TORCH_CHECK(v_cache.scalar_type() == k_cache.scalar_type(), "k/v cache dtype");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D,
              "k_cache [blocks, Hkv, bs, D]");
  TORCH_CHECK(k_cache.stride(3) == 1 && k_cache.stride(2) == D && k_cache.stride(1) == k_cache.size(2) * D,
              "k_cache inner layout");
  TORCH_CHECK(v_cache.sizes() == k_cache.sizes() && v_cache.strides() == k_cache.strides(),
              "v_cache layout");
  llmd_rope_cache(qkv.data_ptr(), qkv.stride(0), positions.data_ptr<int64_t>(),
                  cos_sin.data_ptr<float>(), rot, Hq, Hkv, D, slots.data_ptr<int64_t>(),
                  k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0), k_cache.size(2), T,
                  neox ? 1 : 0, f8 ? 1 : 0, (float)(1.0 / k_scale), (float)(1.0 / v_scale), cur_stream());
}

// The decode QKV projection's split-K partials (mgemm_partials) reduced, rotated and written to the paged
// cache in one kernel: qkv [T, W] receives the projection (Q rotated), K / V go to the cache.
void reduce_rope_cache(torch::Tensor part, int64_t nsplit, torch::Tensor qkv, torch::Tensor positions,
                       torch::Tensor cos_sin, int64_t Hq, int64_t Hkv, int64_t D, torch::Tensor slots,
                       torch::Tensor k_cache, torch::Tensor v_cache, bool neox, double k_scale, double v_scale) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(qkv));
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_INNER(qkv); CHECK_DT(part, at::kFloat);
  CHECK_DT(positions, at::kLong); CHECK_DT(slots, at::kLong); CHECK_DT(cos_sin, at::kFloat);
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) >= (Hq + 2 * Hkv) * D, "reduce_rope_cache: qkv width");
  const int T = qkv.size(0), W = qkv.size(1);
  TORCH_CHECK(part.numel() >= nsplit * (int64_t)T * W, "reduce_rope_cache: partials");
  TORCH_CHECK(positions.numel() == T && slots.numel() == T, "reduce_rope_cache: T mismatch");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.is_contiguous(), "cos_sin 2-D contiguous");
  const int rot = cos_sin.size(1);
  TORCH_CHECK(rot % 16 == 0 && rot <= D && D % 8 == 0, "reduce_rope_cache: rotary dim");
  const bool f8 = is_fp8_cache(k_cache);
  TORCH_CHECK(v_cache.scalar_type() == k_cache.scalar_type(), "k/v cache dtype");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D &&
              k_cache.stride(3) == 1 && k_cache.stride(2) == D && k_cache.stride(1) == k_cache.size(2) * D &&
              v_cache.sizes() == k_cache.sizes() && v_cache.strides() == k_cache.strides(), "k/v cache layout");
  int rc = llmd_reduce_rope_cache(part.data_ptr<float>(), (int)nsplit, W, qkv.data_ptr(), qkv.stride(0),
                                  positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(), rot, Hq, Hkv, D,
                                  slots.data_ptr<int64_t>(), k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0),
                                  k_cache.size(2), T, neox ? 1 : 0, f8 ? 1 : 0, (float)(1.0 / k_scale),
                                  (float)(1.0 / v_scale), cur_stream());
  TORCH_CHECK(rc == 0, "reduce_rope_cache failed: ", rc);
}

// split-K partials of y = x w^T (csrc/ops/mgemm.hip) for a consumer that fuses the reduce; returns nsplit
int64_t mgemm_partials(torch::Tensor x, torch::Tensor w, int64_t wrb, int64_t nsplit, int64_t stages,
                       torch::Tensor part) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_INNER(x); CHECK_INNER(w); CHECK_DT(part, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == x.size(1), "mgemm_partials: shapes");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(part.numel() >= nsplit * (int64_t)M * N, "mgemm_partials: workspace");
  int rc = llmd_mgemm_partials(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, (int)wrb, (int)nsplit,
                               (int)stages, part.data_ptr<float>(), cur_stream());
  TORCH_CHECK(rc >= 2, "mgemm_partials failed: ", rc);
  return rc;
}

void gated_act(torch::Tensor out, torch::Tensor x, int64_t mode, double alpha, double limit) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(out));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_INNER(x); CHECK_INNER(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(0) == out.size(0), "gated_act shape");
  const int F = out.size(1);
  TORCH_CHECK(x.size(1) == 2 * F && F % 8 == 0, "gated_act: x must be [T, 2F], F % 8 == 0");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "16-B aligned rows");
  llmd_gated_act(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), x.size(0), F, (int)mode,
                 (float)alpha, (float)limit, cur_stream());
}

void check_cache(const torch::Tensor& k, const torch::Tensor& v, int64_t Hkv, int64_t D) {
  is_fp8_cache(k);
  TORCH_CHECK(v.scalar_type() == k.scalar_type(), "k/v cache dtype");
  TORCH_CHECK(k.dim() == 4 && k.size(1) == Hkv && k.size(3) == D, "cache [blocks, Hkv, bs, D]");
  TORCH_CHECK(k.stride(3) == 1 && k.stride(2) == D && k.stride(1) == k.size(2) * D,
              "cache inner layout");
  TORCH_CHECK(v.sizes() == k.sizes() && v.strides() == k.strides(), "v_cache layout");
  TORCH_CHECK(k.size(2) > 0 && (k.size(2) & (k.size(2) - 1)) == 0, "KV block size must be a power of two");
}

// q [B, >=Hq*D] (token stride), out [B, Hq*D]
void paged_decode(torch::Tensor out, torch::Tensor q, torch::Tensor k_cache, torch::Tensor v_cache,
                  torch::Tensor block_tables, torch::Tensor seq_lens, int64_t Hq, int64_t Hkv,
                  int64_t D, double scale, int64_t window, c10::optional<torch::Tensor> sinks,
                  int64_t split_size, int64_t nsplit, torch::Tensor part_o, torch::Tensor part_ml,
                  double k_scale, double v_scale, c10::optional<torch::Tensor> cascade, int64_t np,
                  int64_t nslot, c10::optional<torch::Tensor> split_dev) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(out));
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_INNER(q); CHECK_INNER(out);
  check_cache(k_cache, v_cache, Hkv, D);
  CHECK_DT(block_tables, at::kInt); CHECK_DT(seq_lens, at::kInt);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.stride(1) == 1, "block_tables 2-D");
  const int B = q.size(0);
  TORCH_CHECK(seq_lens.numel() == B && block_tables.size(0) >= B, "decode: batch mismatch");
  TORCH_CHECK(Hq % Hkv == 0 && (D == 64 || D == 128), "decode: heads/D");
  TORCH_CHECK(q.size(1) >= Hq * D && out.size(0) >= B && out.size(1) >= Hq * D, "decode: widths");
  TORCH_CHECK(split_size % 64 == 0 && split_size > 0 && nsplit >= 1, "decode: split");
  TORCH_CHECK(q.stride(0) % 8 == 0, "decode: 16-B aligned q rows");
  const float* sk = nullptr;
  if (sinks.has_value()) {
    CHECK_DT(sinks.value(), at::kFloat);
    TORCH_CHECK(sinks->numel() == Hq, "sinks [Hq]");
    sk = sinks->data_ptr<float>();
  }
  // cascade: int32 [sstart(B) | pcount(B) | members(B) | work(nwork x 5)] (ops.cascade_tensors)
  const int *sstart = nullptr, *pcount = nullptr, *members = nullptr, *work = nullptr;
  int nwork = 0;
  if (cascade.has_value()) {
    CHECK_CUDA(cascade.value()); CHECK_DT(cascade.value(), at::kInt);
    const int64_t n = cascade->numel();
    TORCH_CHECK(n >= 3 * (int64_t)B && (n - 3 * (int64_t)B) % 5 == 0, "decode: cascade tensor layout");
    TORCH_CHECK(cascade->is_contiguous(), "decode: cascade tensor contiguous");
    sstart = cascade->data_ptr<int>();
    pcount = sstart + B;
    members = sstart + 2 * B;
    work = sstart + 3 * B;
    nwork = (int)((n - 3 * (int64_t)B) / 5);
    const int64_t G = Hq / Hkv;
    TORCH_CHECK(G <= 16 && 16 % G == 0 && np >= 1 && np <= 3, "decode: cascade needs 16 % G == 0, np in {1,2,3}");
    TORCH_CHECK(np != 3 || (!is_fp8_cache(k_cache) && (G == 4 || G == 8) && k_cache.size(2) >= 8),
                "decode: cascade kernel 3 needs a bf16 cache, G 4 or 8, block size >= 8");
    TORCH_CHECK(nslot > nsplit, "decode: cascade needs prefix slots");
  } else {
    nslot = nsplit;
  }
  // split_dev: int32 [1] on the device = keys per split, overriding split_size (hipGraph
  // replay); the caller keeps split_dev * nsplit >= the longest (suffix) context
  const int* sdev = nullptr;
  if (split_dev.has_value()) {
    CHECK_CUDA(split_dev.value()); CHECK_DT(split_dev.value(), at::kInt);
    TORCH_CHECK(split_dev->numel() >= 1, "decode: split_dev [1]");
    sdev = split_dev->data_ptr<int>();
  }
  if (nsplit > 1 || nwork > 0) {
    CHECK_DT(part_o, at::kFloat); CHECK_DT(part_ml, at::kFloat);
    TORCH_CHECK(part_o.numel() >= (int64_t)B * Hq * nslot * D &&
                    part_ml.numel() >= (int64_t)B * Hq * nslot * 2, "decode workspace too small");
  }
  // the host must guarantee ctx <= nsplit*split_size (checked by the caller, no sync here)
  int rc = llmd_paged_decode(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                             k_cache.stride(0), k_cache.size(2), block_tables.data_ptr<int>(),
                             block_tables.stride(0), seq_lens.data_ptr<int>(), B, Hq, Hkv, D,
                             (float)scale, (int)window, sk, split_size, nsplit, out.data_ptr(),
                             out.stride(0), (nsplit > 1 || nwork > 0) ? part_o.data_ptr<float>() : nullptr,
                             (nsplit > 1 || nwork > 0) ? part_ml.data_ptr<float>() : nullptr,
                             is_fp8_cache(k_cache) ? 1 : 0, (float)k_scale, (float)v_scale, sstart, pcount,
                             members, work, nwork, (int)np, (int)nslot, sdev, cur_stream());
  TORCH_CHECK(rc == 0, "paged_decode: unsupported head dim / cascade config, rc=", rc);
}

// MLA (absorbed form): q [R, H*576], cache [blocks, bs, 576] (block stride free),
// out [R, H*512]; row r attends to keys [0, row_len[r]) of sequence row_seq[r].
void mla_attention(torch::Tensor out, torch::Tensor q, torch::Tensor cache, torch::Tensor block_tables,
                   torch::Tensor row_seq, torch::Tensor row_len, int64_t H, double scale, int64_t split_size,
                   int64_t nsplit, torch::Tensor part_o, torch::Tensor part_ml, double kv_scale,
                   c10::optional<torch::Tensor> split_dev) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(out));
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_INNER(q); CHECK_INNER(out);
  const bool f8 = is_fp8_cache(cache);
  const int* sdev = nullptr;  // int32 [1] keys per split (hipGraph replay), overrides split_size
  if (split_dev.has_value()) {
    CHECK_CUDA(split_dev.value()); CHECK_DT(split_dev.value(), at::kInt);
    sdev = split_dev->data_ptr<int>();
  }
  CHECK_DT(block_tables, at::kInt); CHECK_DT(row_seq, at::kInt); CHECK_DT(row_len, at::kInt);
  TORCH_CHECK(cache.dim() == 3 && cache.size(2) == 576 && cache.stride(2) == 1 && cache.stride(1) == 576,
              "mla cache [blocks, bs, 576] with contiguous rows");
  TORCH_CHECK(cache.size(1) > 0 && (cache.size(1) & (cache.size(1) - 1)) == 0, "MLA block size must be a power of two");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.stride(1) == 1, "block_tables 2-D");
  const int R = q.size(0);
  TORCH_CHECK(row_seq.numel() == R && row_len.numel() == R, "mla: rows mismatch");
  TORCH_CHECK(q.size(1) >= H * 576 && out.size(0) >= R && out.size(1) >= H * 512, "mla: widths");
  TORCH_CHECK(q.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "mla: 16-B aligned rows");
  TORCH_CHECK(split_size % 64 == 0 && split_size > 0 && nsplit >= 1, "mla: split");
  if (nsplit > 1) {
    CHECK_DT(part_o, at::kFloat); CHECK_DT(part_ml, at::kFloat);
    TORCH_CHECK(part_o.numel() >= (int64_t)R * H * nsplit * 512 && part_ml.numel() >= (int64_t)R * H * nsplit * 2,
                "mla workspace too small");
  }
  int rc = llmd_mla_attention(q.data_ptr(), q.stride(0), cache.data_ptr(), cache.stride(0), cache.size(1),
                              block_tables.data_ptr<int>(), block_tables.stride(0), row_seq.data_ptr<int>(),
                              row_len.data_ptr<int>(), R, H, (float)scale, split_size, nsplit, out.data_ptr(),
                              out.stride(0), nsplit > 1 ? part_o.data_ptr<float>() : nullptr,
                              nsplit > 1 ? part_ml.data_ptr<float>() : nullptr, f8 ? 1 : 0, (float)kv_scale,
                              sdev, cur_stream());
  TORCH_CHECK(rc == 0, "mla_attention failed: ", rc);
}

void mla_rope_cache(torch::Tensor q, torch::Tensor q_lat, torch::Tensor kv_c, torch::Tensor k_pe,
                    torch::Tensor positions, torch::Tensor cos_sin, int64_t H, torch::Tensor slots,
                    torch::Tensor cache, double kv_scale) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(q));
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(q_lat); CHECK_BF16(kv_c); CHECK_BF16(k_pe);
  const bool f8 = is_fp8_cache(cache);
  TORCH_CHECK(kv_scale > 0, "mla_rope: kv_scale must be positive");
  CHECK_INNER(q); CHECK_INNER(q_lat); CHECK_INNER(kv_c); CHECK_INNER(k_pe);
  CHECK_DT(positions, at::kLong); CHECK_DT(slots, at::kLong); CHECK_DT(cos_sin, at::kFloat);
  const int T = q.size(0);
  TORCH_CHECK(q.size(1) >= H * 192 && q_lat.size(0) >= T && q_lat.size(1) >= H * 576, "mla_rope: q widths");
  TORCH_CHECK(kv_c.size(0) >= T && kv_c.size(1) == 512 && k_pe.size(0) >= T && k_pe.size(1) == 64,
              "mla_rope: kv_c [T,512], k_pe [T,64]");
  TORCH_CHECK(kv_c.stride(0) % 8 == 0, "mla_rope: 16-B aligned kv_c rows");
  TORCH_CHECK(positions.numel() >= T && slots.numel() >= T, "mla_rope: positions/slots");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == 64 && cos_sin.is_contiguous(), "mla_rope: cos_sin [P,64]");
  TORCH_CHECK(cache.dim() == 3 && cache.size(2) == 576 && cache.stride(1) == 576, "mla_rope: cache [blocks,bs,576]");
  int rc = llmd_mla_rope_cache(q.data_ptr(), q.stride(0), q_lat.data_ptr(), q_lat.stride(0), kv_c.data_ptr(),
                               kv_c.stride(0), k_pe.data_ptr(), k_pe.stride(0), positions.data_ptr<int64_t>(),
                               cos_sin.data_ptr<float>(), T, H, slots.data_ptr<int64_t>(), cache.data_ptr(),
                               cache.stride(0), cache.size(1), f8 ? 1 : 0, (float)(1.0 / kv_scale), cur_stream());
  TORCH_CHECK(rc == 0, "mla_rope_cache failed: ", rc);
}

// y[t] += B[slot[t]] @ (A[slot[t]] @ x[t]); A [S, R, in], B [S, out, R] bf16, slot [T] int32
void lora_bgmv(torch::Tensor y, torch::Tensor x, torch::Tensor A, torch::Tensor B, torch::Tensor slot,
               torch::Tensor h) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(y); CHECK_BF16(A); CHECK_BF16(B); CHECK_INNER(x); CHECK_INNER(y);
  CHECK_DT(slot, at::kInt); CHECK_DT(h, at::kFloat);
  TORCH_CHECK(A.dim() == 3 && B.dim() == 3 && A.is_contiguous() && B.is_contiguous(), "lora: A [S,R,in], B [S,out,R]");
  const int T = x.size(0), R = A.size(1), in = A.size(2), out = B.size(1);
  TORCH_CHECK(B.size(0) == A.size(0) && B.size(2) == R && R <= 128, "lora: slot/rank mismatch");
  TORCH_CHECK(x.size(1) == in && y.size(0) == T && y.size(1) == out && slot.numel() >= T, "lora: shapes");
  TORCH_CHECK(in % 8 == 0 && in <= 32768 && x.stride(0) % 8 == 0, "lora: in dim");
  TORCH_CHECK(h.numel() >= (int64_t)T * R, "lora: workspace");
  int rc = llmd_lora_bgmv(x.data_ptr(), x.stride(0), A.data_ptr(), B.data_ptr(), T, R, in, out, slot.data_ptr<int>(),
                          h.data_ptr<float>(), y.data_ptr(), y.stride(0), cur_stream());
  TORCH_CHECK(rc == 0, "lora_bgmv failed: ", rc);
}

// y [M, N] = x [M, K] . w [N, K]^T for M <= 64 (decode GEMMs): rb row blocks of
// 16 per workgroup, nsplit-way split-K, occ workgroups per CU (ops.skinny_plan)
void skinny_gemm(torch::Tensor y, torch::Tensor x, torch::Tensor w, int64_t rb, int64_t nsplit, int64_t occ,
                 torch::Tensor part) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(y);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "skinny_gemm: 2-D operands");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && w.size(1) == K && K % 256 == 0, "skinny_gemm: M <= 64, K % 256 == 0");
  TORCH_CHECK(N % 4 == 0, "skinny_gemm: N % 4 == 0");
  TORCH_CHECK(y.size(0) == M && y.size(1) == N, "skinny_gemm: output shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && y.stride(0) % 4 == 0, "skinny_gemm: row alignment");
  TORCH_CHECK(llmd_dgemm_supported(M, (int)rb, (int)occ), "skinny_gemm: no kernel for rb=", rb, " occ=", occ);
  if (nsplit > 1) {
    CHECK_DT(part, at::kFloat);
    TORCH_CHECK(part.numel() >= nsplit * (int64_t)M * N, "skinny_gemm: workspace");
  }
  int rc = llmd_skinny_gemm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, (int)rb, (int)nsplit,
                            (int)occ, y.data_ptr(), y.stride(0), nsplit > 1 ? part.data_ptr<float>() : nullptr,
                            cur_stream());
  TORCH_CHECK(rc == 0, "skinny_gemm failed: ", rc);
}

extern "C" int llmd_mla_v2_shape(int R, int fp8);
int64_t mla_v2_shape(int64_t R, bool fp8) { return llmd_mla_v2_shape((int)R, fp8 ? 1 : 0); }

bool skinny_supported(int64_t M, int64_t rb, int64_t occ) { return llmd_dgemm_supported((int)M, (int)rb, (int)occ); }

// y [M, N] = x [M, K] . w [N, K]^T for 33 <= M <= 256 (decode batches of a P/D
// decode replica): LDS-DMA staged tiles of 64 wrb W rows x all M, nsplit-way
// split-K, 3- or 4-stage ring (csrc/ops/mgemm.hip)
// Split-K fixup counters of mgemm (csrc/ops/mgemm.hip): per device 256 slabs of 1024 zeroed ints, handed
// out round-robin so kernels in flight on different streams (DBO, TP overlap) never share a slab; each
// launch leaves its slab zeroed. Created outside stream capture (a capture before the first eager call
// falls back to the reduce kernel). Opt-in (LLMD_MGEMM_FIXUP=1): with agent-scope fences in every
// workgroup it measured slower than the reduce launch (profiles/decode_r5.txt).
int* mgemm_counters(const torch::Device& d, int64_t tiles) {
  static const bool on = [] {
    const char* e = getenv("LLMD_MGEMM_FIXUP");
    return e && e[0] == '1';
  }();
  if (!on || tiles > 1024) return nullptr;
  static std::mutex mu;
  static std::map<int, torch::Tensor> pools;
  static std::map<int, uint32_t> next;
  std::lock_guard<std::mutex> g(mu);
  auto& t = pools[d.index()];
  if (!t.defined()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(cur_stream(), &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    t = torch::zeros({256 * 1024}, torch::dtype(torch::kInt32).device(d));
  }
  const uint32_t i = next[d.index()]++ % 256;
  return t.data_ptr<int>() + (int64_t)i * 1024;
}

void mgemm(torch::Tensor y, torch::Tensor x, torch::Tensor w, int64_t wrb, int64_t nsplit, int64_t stages,
           torch::Tensor part) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(y);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "mgemm: 2-D operands");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 256 && w.size(1) == K && K % 64 == 0, "mgemm: M <= 256, K % 64 == 0");
  TORCH_CHECK(N % 4 == 0 && y.size(0) == M && y.size(1) == N, "mgemm: output shape / N % 4");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && y.stride(0) % 4 == 0, "mgemm: row alignment");
  TORCH_CHECK(llmd_mgemm_lds(M, (int)wrb, (int)stages) > 0, "mgemm: no kernel for wrb=", wrb, " stages=", stages);
  if (nsplit > 1) {
    CHECK_DT(part, at::kFloat);
    TORCH_CHECK(part.numel() >= nsplit * (int64_t)M * N, "mgemm: workspace");
  }
  int rc = llmd_mgemm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, (int)wrb, (int)nsplit,
                      (int)stages, y.data_ptr(), y.stride(0), nsplit > 1 ? part.data_ptr<float>() : nullptr,
                      nsplit > 1 ? mgemm_counters(y.device(), (N + 64 * wrb - 1) / (64 * wrb)) : nullptr,
                      cur_stream());
  TORCH_CHECK(rc == 0, "mgemm failed: ", rc);
}

// out = rmsnorm(residual + x w^T) * gamma with residual updated in place: the decode step's o / down
// projection on the split-K medium-M GEMM with the residual-add + RMSNorm in its reduce (csrc/ops/mgemm.hip)
void mgemm_add_rmsnorm(torch::Tensor out, torch::Tensor x, torch::Tensor w, int64_t wrb, int64_t nsplit,
                       int64_t stages, torch::Tensor part, torch::Tensor residual, torch::Tensor gamma, double eps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(out));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_BF16(residual); CHECK_BF16(gamma);
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out); CHECK_INNER(residual); CHECK_DT(part, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2 && residual.dim() == 2, "mgemm_add_rmsnorm: 2-D operands");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 128 && w.size(1) == K && K % 64 == 0 && N % 8 == 0, "mgemm_add_rmsnorm: shapes");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N && residual.size(0) == M && residual.size(1) == N &&
              gamma.numel() == N, "mgemm_add_rmsnorm: output / residual / gamma shape");
  TORCH_CHECK(nsplit > 1 && part.numel() >= nsplit * (int64_t)M * N, "mgemm_add_rmsnorm: split-K workspace");
  int rc = llmd_mgemm_add_rmsnorm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, (int)wrb,
                                  (int)nsplit, (int)stages, part.data_ptr<float>(), residual.data_ptr(),
                                  residual.stride(0), gamma.data_ptr(), (float)eps, out.data_ptr(), out.stride(0),
                                  cur_stream());
  TORCH_CHECK(rc == 0, "mgemm_add_rmsnorm failed: ", rc);
}

// y [M, N] = x [M, K] . w [N, K]^T for prefill-sized M on the 256 x 256 LDS-DMA MFMA
// GEMM (csrc/ops/pgemm.hip); epi 1 = fused SiLU-and-mul over gate/up columns interleaved
// per 256-column tile, epi 3 = the same on the plain [gate; up] weight (variants 3-5); y is
// then [M, N / 2]
// variant 1 with split_k: a mostly idle last wave of tiles runs split over K into an fp32
// workspace (allocated here from the caching allocator) and is reduced by a second kernel
void pgemm(torch::Tensor y, torch::Tensor x, torch::Tensor w, int64_t epi, int64_t variant, bool split_k) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(y);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "pgemm: 2-D operands");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 256 == 0, "pgemm: N % 256 == 0, K % 64 == 0");
  TORCH_CHECK(y.size(0) == M && y.size(1) == ((epi == 1 || epi == 3) ? N / 2 : N), "pgemm: output shape");
  TORCH_CHECK(epi != 3 || (variant >= 3 && variant <= 6), "pgemm: epi 3 (SiLU on the [gate; up] weight) needs variant 3-6");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && y.stride(0) % 8 == 0, "pgemm: 16-B row alignment");
  torch::Tensor ws;
  const int64_t wsb = split_k ? llmd_pgemm_ws_bytes((int)M, (int)N, (int)K, (int)epi, (int)variant) : 0;
  if (wsb > 0) ws = torch::empty({wsb / 4}, x.options().dtype(torch::kFloat));
  int rc = llmd_pgemm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), y.data_ptr(), y.stride(0), (int)M,
                      (int)N, (int)K, (int)epi, (int)variant, wsb > 0 ? ws.data_ptr() : nullptr, cur_stream());
  TORCH_CHECK(rc == 0, "pgemm failed: ", rc);
}

// y = (xs . xq) (ws . wq)^T for prefill-sized M on the fp8 256 x 256 LDS-DMA GEMM (csrc/ops/pgemm8.hip,
// v_mfma_scale_f32_16x16x128_f8f6f4): xq [M, K] / wq [N, K] e4m3fn, xs [M] or [M, 1] and ws [N] or
// [1, N] fp32; epi 3 = silu(gate) * up on wq = [gate; up], y [M, N / 2]
void pgemm_fp8(torch::Tensor y, torch::Tensor xq, torch::Tensor xs, torch::Tensor wq, torch::Tensor ws, int64_t epi,
               bool split_k, bool persistent) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(xq); CHECK_BF16(y); CHECK_INNER(xq); CHECK_INNER(wq); CHECK_INNER(y);
  TORCH_CHECK(xq.scalar_type() == at::kFloat8_e4m3fn && wq.scalar_type() == at::kFloat8_e4m3fn, "pgemm_fp8: e4m3fn");
  TORCH_CHECK(xs.scalar_type() == at::kFloat && ws.scalar_type() == at::kFloat, "pgemm_fp8: fp32 scales");
  TORCH_CHECK(xs.is_contiguous() && ws.is_contiguous(), "pgemm_fp8: contiguous scales");
  TORCH_CHECK(xq.dim() == 2 && wq.dim() == 2 && y.dim() == 2, "pgemm_fp8: 2-D operands");
  const int64_t M = xq.size(0), K = xq.size(1), N = wq.size(0);
  TORCH_CHECK(wq.size(1) == K && K % 128 == 0 && N % 256 == 0, "pgemm_fp8: N % 256 == 0, K % 128 == 0");
  TORCH_CHECK(xs.numel() == M && ws.numel() == N, "pgemm_fp8: per-token / per-channel scales");
  TORCH_CHECK(epi == 0 || epi == 3, "pgemm_fp8: epi 0 or 3");
  TORCH_CHECK(y.size(0) == M && y.size(1) == (epi == 3 ? N / 2 : N), "pgemm_fp8: output shape");
  TORCH_CHECK(xq.stride(0) % 16 == 0 && wq.stride(0) % 16 == 0 && y.stride(0) % 8 == 0, "pgemm_fp8: 16-B rows");
  // split_k: a mostly idle last wave of tiles runs split over K into an fp32 workspace
  torch::Tensor wsp;
  const int64_t wsb = (split_k && !(persistent && epi == 0)) ? llmd_pgemm_fp8_ws_bytes((int)M, (int)N, (int)K, (int)epi)
                                                            : 0;
  if (wsb > 0) wsp = torch::empty({wsb / 4}, xs.options());
  int rc = llmd_pgemm_fp8(xq.data_ptr(), xq.stride(0), xs.data_ptr<float>(), wq.data_ptr(), wq.stride(0),
                          ws.data_ptr<float>(), y.data_ptr(), y.stride(0), (int)M, (int)N, (int)K, (int)epi,
                          wsb > 0 ? wsp.data_ptr() : nullptr, persistent ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "pgemm_fp8 failed: ", rc);
}

// y [M, F] = silu(x wg^T) * (x wu^T), w = [gate; up] [2F, K] (mgemm ACT form, whole K per workgroup)
void mgemm_silu(torch::Tensor y, torch::Tensor x, torch::Tensor w, int64_t wrb, int64_t stages) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(y);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "mgemm_silu: 2-D operands");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 256 && w.size(1) == K && K % 64 == 0 && N % 8 == 0, "mgemm_silu: shapes");
  TORCH_CHECK(y.size(0) == M && y.size(1) == N / 2, "mgemm_silu: y [M, N / 2]");
  int rc = llmd_mgemm_silu(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), M, N, K, (int)wrb, (int)stages,
                           y.data_ptr(), y.stride(0), cur_stream());
  TORCH_CHECK(rc == 0, "mgemm_silu failed: ", rc);
}

// fp8 W8A8 form: xq [M, K] e4m3fn with per-token scales xs [M, 1], wq [N, K] e4m3fn with
// per-channel scales ws [1, N] (ops.fp8_linear's operands); K % 128 == 0
void mgemm_fp8(torch::Tensor y, torch::Tensor xq, torch::Tensor xs, torch::Tensor wq, torch::Tensor ws, int64_t wrb,
               int64_t nsplit, int64_t stages, torch::Tensor part) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  CHECK_CUDA(xq); CHECK_BF16(y); CHECK_INNER(xq); CHECK_INNER(wq); CHECK_INNER(y);
  TORCH_CHECK(xq.scalar_type() == at::kFloat8_e4m3fn && wq.scalar_type() == at::kFloat8_e4m3fn, "mgemm_fp8: e4m3fn");
  CHECK_DT(xs, at::kFloat); CHECK_DT(ws, at::kFloat);
  TORCH_CHECK(xq.dim() == 2 && wq.dim() == 2 && y.dim() == 2, "mgemm_fp8: 2-D operands");
  const int M = xq.size(0), K = xq.size(1), N = wq.size(0);
  TORCH_CHECK(M >= 1 && M <= 256 && wq.size(1) == K && K % 128 == 0, "mgemm_fp8: M <= 256, K % 128 == 0");
  TORCH_CHECK(N % 4 == 0 && y.size(0) == M && y.size(1) == N, "mgemm_fp8: output shape / N % 4");
  TORCH_CHECK(xs.is_contiguous() && xs.numel() == M && ws.is_contiguous() && ws.numel() == N, "mgemm_fp8: scales");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(ws.data_ptr()) % 16 == 0, "mgemm_fp8: 16-B aligned weight scales");
  TORCH_CHECK(xq.stride(0) % 16 == 0 && wq.stride(0) % 16 == 0 && y.stride(0) % 4 == 0, "mgemm_fp8: row alignment");
  TORCH_CHECK(llmd_mgemm_lds(M, (int)wrb, (int)stages) > 0, "mgemm_fp8: no kernel for wrb=", wrb, " stages=", stages);
  if (nsplit > 1) {
    CHECK_DT(part, at::kFloat);
    TORCH_CHECK(part.numel() >= nsplit * (int64_t)M * N, "mgemm_fp8: workspace");
  }
  int rc = llmd_mgemm_fp8(xq.data_ptr(), xq.stride(0), xs.data_ptr<float>(), wq.data_ptr(), wq.stride(0),
                          ws.data_ptr<float>(), M, N, K, (int)wrb, (int)nsplit, (int)stages, y.data_ptr(), y.stride(0),
                          nsplit > 1 ? part.data_ptr<float>() : nullptr,
                          nsplit > 1 ? mgemm_counters(y.device(), (N + 64 * wrb - 1) / (64 * wrb)) : nullptr,
                          cur_stream());
  TORCH_CHECK(rc == 0, "mgemm_fp8 failed: ", rc);
}

extern "C" int llmd_kv_dequant_gather(const void*, const void*, int64_t, const int*, int, int, int, void*, void*,
                                      hipStream_t);

// fp8 paged K/V blocks of a block table -> dense bf16 copies kd / vd [entries, Hkv, bs, D] (attn_prefill.hip)
void kv_dequant_gather(torch::Tensor k_cache, torch::Tensor v_cache, torch::Tensor block_tables, torch::Tensor kd,
                       torch::Tensor vd) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(k_cache));
  CHECK_CUDA(k_cache); CHECK_DT(k_cache, at::kFloat8_e4m3fn); CHECK_DT(v_cache, at::kFloat8_e4m3fn);
  CHECK_BF16(kd); CHECK_BF16(vd); CHECK_DT(block_tables, at::kInt);
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.sizes() == k_cache.sizes() && v_cache.stride(0) == k_cache.stride(0),
              "caches [blocks, Hkv, bs, D], same layout");
  const int64_t per = k_cache.size(1) * k_cache.size(2) * k_cache.size(3);
  TORCH_CHECK(k_cache.stride(3) == 1 && k_cache.stride(2) == k_cache.size(3) &&
              k_cache.stride(1) == k_cache.size(2) * k_cache.size(3), "a block's [Hkv, bs, D] contiguous");
  TORCH_CHECK(block_tables.is_contiguous() && kd.is_contiguous() && vd.is_contiguous() &&
              kd.numel() == block_tables.numel() * per && vd.numel() == kd.numel(), "kd / vd [entries, Hkv, bs, D]");
  const int rc = llmd_kv_dequant_gather(k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0),
                                        block_tables.data_ptr<int>(), (int)block_tables.numel(),
                                        (int)k_cache.size(0), (int)per, kd.data_ptr(), vd.data_ptr(), cur_stream());
  TORCH_CHECK(rc == 0, "kv_dequant_gather failed: ", rc);
}

void paged_prefill(torch::Tensor out, torch::Tensor q, torch::Tensor k_cache,
                   torch::Tensor v_cache, torch::Tensor block_tables, torch::Tensor q_start,
                   torch::Tensor q_len, torch::Tensor ctx_len, torch::Tensor items, int64_t Hq,
                   int64_t Hkv, int64_t D, double scale, int64_t window,
                   c10::optional<torch::Tensor> sinks, double k_scale, double v_scale) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(out));
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_INNER(q); CHECK_INNER(out);
  check_cache(k_cache, v_cache, Hkv, D);
  CHECK_DT(block_tables, at::kInt); CHECK_DT(q_start, at::kInt); CHECK_DT(q_len, at::kInt);
  CHECK_DT(ctx_len, at::kInt); CHECK_DT(items, at::kInt);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.stride(1) == 1, "block_tables 2-D");
  TORCH_CHECK(items.dim() == 2 && items.size(1) == 2 && items.is_contiguous(), "items [n, 2]");
  TORCH_CHECK(Hq % Hkv == 0 && (D == 64 || D == 128), "prefill: heads/D");
  TORCH_CHECK(q.size(1) >= Hq * D && out.size(1) >= Hq * D && out.size(0) >= q.size(0), "widths");
  TORCH_CHECK(q.stride(0) % 8 == 0, "prefill: 16-B aligned q rows");
  const float* sk = nullptr;
  if (sinks.has_value()) {
    CHECK_DT(sinks.value(), at::kFloat);
    TORCH_CHECK(sinks->numel() == Hq, "sinks [Hq]");
    sk = sinks->data_ptr<float>();
  }
  int rc = llmd_paged_prefill(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                              k_cache.stride(0), k_cache.size(2), block_tables.data_ptr<int>(),
                              block_tables.stride(0), q_start.data_ptr<int>(),
                              q_len.data_ptr<int>(), ctx_len.data_ptr<int>(),
                              items.data_ptr<int>(), items.size(0), Hq, Hkv, D, (float)scale,
                              (int)window, sk, out.data_ptr(), out.stride(0), is_fp8_cache(k_cache) ? 1 : 0,
                              (float)k_scale, (float)v_scale, cur_stream());
  TORCH_CHECK(rc == 0, "paged_prefill: unsupported head dim");
}

void sample(torch::Tensor logits, c10::optional<torch::Tensor> temps,
            c10::optional<torch::Tensor> seeds, torch::Tensor out_ids,
            c10::optional<torch::Tensor> out_logprob) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(logits));
  CHECK_CUDA(logits); CHECK_INNER(logits);
  TORCH_CHECK(logits.dim() == 2, "logits 2-D");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "logits bf16/f32");
  const int B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(logits.stride(0) % (bf ? 8 : 4) == 0, "16-B aligned logits rows");
  CHECK_DT(out_ids, at::kLong);
  TORCH_CHECK(out_ids.numel() >= B, "out_ids");
  const float* t = nullptr;
  const int64_t* s = nullptr;
  float* lp = nullptr;
  if (temps.has_value()) { CHECK_DT(temps.value(), at::kFloat); TORCH_CHECK(temps->numel() >= B); t = temps->data_ptr<float>(); }
  if (seeds.has_value()) { CHECK_DT(seeds.value(), at::kLong); TORCH_CHECK(seeds->numel() >= B); s = seeds->data_ptr<int64_t>(); }
  if (out_logprob.has_value()) { CHECK_DT(out_logprob.value(), at::kFloat); lp = out_logprob->data_ptr<float>(); }
  // small batches: each row split over several workgroups (partials merged by a second kernel)
  const int nsp = llmd_sample_splits(B, V);
  at::Tensor part;
  if (nsp > 1) part = at::empty({(int64_t)B * nsp * 4}, logits.options().dtype(at::kFloat));
  llmd_sample(logits.data_ptr(), logits.stride(0), B, V, bf ? 1 : 0, t, s,
              out_ids.data_ptr<int64_t>(), lp, nsp > 1 ? part.data_ptr<float>() : nullptr, nsp, cur_stream());
}

void topk_topp_mask(torch::Tensor logits, c10::optional<torch::Tensor> topk,
                    c10::optional<torch::Tensor> topp, c10::optional<torch::Tensor> temps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(logits));
  CHECK_CUDA(logits); CHECK_DT(logits, at::kFloat); CHECK_INNER(logits);
  const int B = logits.size(0), V = logits.size(1);
  const int* k = nullptr;
  const float* p = nullptr;
  const float* t = nullptr;
  if (topk.has_value()) { CHECK_DT(topk.value(), at::kInt); TORCH_CHECK(topk->numel() >= B); k = topk->data_ptr<int>(); }
  if (topp.has_value()) { CHECK_DT(topp.value(), at::kFloat); TORCH_CHECK(topp->numel() >= B); p = topp->data_ptr<float>(); }
  if (temps.has_value()) { CHECK_DT(temps.value(), at::kFloat); TORCH_CHECK(temps->numel() >= B); t = temps->data_ptr<float>(); }
  llmd_topk_topp_mask(logits.data_ptr<float>(), logits.stride(0), B, V, k, p, t, cur_stream());
}

// ---------------------------------------------------------------- kvx
// dst/src are base addresses of the two KV pools (src may be an IPC-mapped peer pointer)
void kvx_copy_blocks(torch::Tensor dst, int64_t src_ptr, int64_t dst_stride, int64_t src_stride,
                     torch::Tensor pairs, torch::Tensor segs, int64_t max_seg_bytes, int64_t engine) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(dst));
  CHECK_CUDA(dst); CHECK_CUDA(pairs); CHECK_CUDA(segs);
  CHECK_DT(pairs, at::kInt); CHECK_DT(segs, at::kLong);
  TORCH_CHECK(pairs.is_contiguous() && pairs.dim() == 2 && pairs.size(1) == 2, "pairs [n,2] int32");
  TORCH_CHECK(segs.is_contiguous() && segs.dim() == 2 && segs.size(1) == 3, "segs [m,3] int64");
  TORCH_CHECK(src_ptr != 0, "null source pool");
  int rc = llmd_kvx_copy_blocks2(dst.data_ptr(), (const void*)src_ptr, dst_stride, src_stride,
                                 pairs.data_ptr<int>(), pairs.size(0), segs.data_ptr<int64_t>(),
                                 segs.size(0), max_seg_bytes, (int)engine, cur_stream());
  TORCH_CHECK(rc == 0, "kvx_copy_blocks failed: ", rc);
}

void kvx_dma_blocks(torch::Tensor dst, int64_t src_ptr, int64_t dst_stride, int64_t src_stride,
                    torch::Tensor pairs_cpu, int64_t block_bytes) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(dst));
  CHECK_CUDA(dst); CHECK_DT(pairs_cpu, at::kInt);
  TORCH_CHECK(!pairs_cpu.is_cuda() && pairs_cpu.is_contiguous() && pairs_cpu.size(1) == 2, "pairs cpu [n,2]");
  int rc = llmd_kvx_dma_blocks(dst.data_ptr(), (const void*)src_ptr, dst_stride, src_stride,
                               pairs_cpu.data_ptr<int>(), pairs_cpu.size(0), block_bytes, cur_stream());
  TORCH_CHECK(rc == 0, "kvx_dma_blocks failed: ", rc);
}

py::tuple kvx_ipc_export(torch::Tensor t) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(t));
  CHECK_CUDA(t);
  std::string h(llmd_kvx_handle_size(), '\0');
  int64_t off = 0;
  int rc = llmd_kvx_ipc_export(t.data_ptr(), h.data(), &off);
  TORCH_CHECK(rc == 0, "hipIpcGetMemHandle failed: ", rc);
  return py::make_tuple(py::bytes(h), off);
}

int64_t kvx_ipc_open(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK((int)h.size() == llmd_kvx_handle_size(), "bad IPC handle size");
  void* p = nullptr;
  int rc = llmd_kvx_ipc_open(h.data(), &p);
  TORCH_CHECK(rc == 0, "hipIpcOpenMemHandle failed: ", rc);
  return (int64_t)p;
}

void kvx_ipc_close(int64_t p) { llmd_kvx_ipc_close((void*)p); }

int64_t vmm_granularity(int64_t device) {
  size_t g = 0;
  int rc = llmd_vmm_granularity((int)device, &g);
  TORCH_CHECK(rc == 0, "hipMemGetAllocationGranularity failed: ", rc);
  return (int64_t)g;
}

// Chunked VMM pool as one uint8 tensor + one exported dmabuf fd per chunk.
py::tuple vmm_pool(int64_t device, int64_t chunk_bytes, int64_t n_chunks) {
  TORCH_CHECK(chunk_bytes > 0 && n_chunks > 0, "vmm_pool: bad size");
  const c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  auto handles = std::make_shared<std::vector<uint64_t>>(n_chunks);
  void* base = nullptr;
  int rc = llmd_vmm_alloc((int)device, (size_t)chunk_bytes, (int)n_chunks, &base, handles->data());
  TORCH_CHECK(rc == 0, "vmm alloc failed: ", rc);
  std::vector<int> fds(n_chunks, -1);
  for (int64_t i = 0; i < n_chunks; ++i) {
    rc = llmd_vmm_export_fd((*handles)[i], &fds[i]);
    TORCH_CHECK(rc == 0, "hipMemExportToShareableHandle failed: ", rc);
  }
  const size_t cb = (size_t)chunk_bytes;
  const int nc = (int)n_chunks;
  auto t = torch::from_blob(
      base, {chunk_bytes * n_chunks},
      [handles, cb, nc](void* p) { llmd_vmm_free(p, cb, nc, handles->data()); },
      torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, (c10::DeviceIndex)device));
  py::list pyfds;
  for (int fd : fds) pyfds.append(fd);
  return py::make_tuple(t, pyfds);
}

struct Imported { size_t chunk; std::vector<uint64_t> handles; };
std::map<int64_t, Imported>& imported() { static std::map<int64_t, Imported> m; return m; }

int64_t vmm_import(std::vector<int64_t> fds, int64_t chunk_bytes, int64_t device) {
  const c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  std::vector<int> f(fds.begin(), fds.end());
  Imported im{(size_t)chunk_bytes, std::vector<uint64_t>(f.size())};
  void* base = nullptr;
  int rc = llmd_vmm_import(f.data(), (int)f.size(), (size_t)chunk_bytes, (int)device, &base, im.handles.data());
  TORCH_CHECK(rc == 0, "vmm import failed: ", rc);
  imported()[(int64_t)base] = std::move(im);
  return (int64_t)base;
}

void vmm_release(int64_t base) {
  auto it = imported().find(base);
  TORCH_CHECK(it != imported().end(), "vmm_release: unknown base");
  llmd_vmm_free((void*)base, it->second.chunk, (int)it->second.handles.size(), it->second.handles.data());
  imported().erase(it);
}

// ---------------------------------------------------------------- MoE
void moe_topk(torch::Tensor logits, int64_t k, int64_t scoring, c10::optional<torch::Tensor> bias,
              int64_t n_group, int64_t topk_group, bool renorm, double routed_scale, torch::Tensor ids,
              torch::Tensor wts) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(logits));
  CHECK_CUDA(logits); CHECK_DT(logits, at::kFloat);
  TORCH_CHECK(logits.is_contiguous() && logits.dim() == 2, "logits [T, E] contiguous f32");
  const int T = logits.size(0), E = logits.size(1);
  TORCH_CHECK(E <= 512 && k >= 1 && k <= 16 && k <= E, "moe_topk: E <= 512, 1 <= k <= 16");
  TORCH_CHECK(n_group <= 64 && (n_group <= 1 || E % n_group == 0), "moe_topk groups");
  CHECK_DT(ids, at::kInt); CHECK_DT(wts, at::kFloat);
  TORCH_CHECK(ids.numel() >= (int64_t)T * k && wts.numel() >= (int64_t)T * k, "moe_topk outputs");
  const float* b = nullptr;
  if (bias.has_value()) { CHECK_DT(bias.value(), at::kFloat); TORCH_CHECK(bias->numel() == E); b = bias->data_ptr<float>(); }
  llmd_moe_topk(logits.data_ptr<float>(), T, E, k, scoring, b, n_group, topk_group, renorm ? 1 : 0,
                (float)routed_scale, ids.data_ptr<int>(), wts.data_ptr<float>(), cur_stream());
}

void moe_align(torch::Tensor ids, int64_t E, torch::Tensor sorted_ids, torch::Tensor tile_expert,
               torch::Tensor expert_offsets, torch::Tensor total_p, torch::Tensor inv, int64_t tile_m) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(ids));
  CHECK_CUDA(ids); CHECK_DT(ids, at::kInt); CHECK_DT(sorted_ids, at::kInt); CHECK_DT(tile_expert, at::kInt);
  const int n = ids.numel();
  const int bm = tile_m > 0 ? (int)tile_m : llmd_moe_gemm_tile_m();
  TORCH_CHECK(bm == llmd_moe_gemm_tile_m() || bm == llmd_moe_gemm3_tile_m() || bm == 192, "moe_align: tile_m");
  const int max_p = sorted_ids.numel();
  TORCH_CHECK(max_p % bm == 0 && max_p >= n + E * (bm - 1), "sorted_ids too small");
  TORCH_CHECK(tile_expert.numel() >= max_p / bm && expert_offsets.numel() >= E + 1 && inv.numel() >= n,
              "moe_align buffers");
  TORCH_CHECK(E <= 4096, "too many experts");
  llmd_moe_align(ids.data_ptr<int>(), n, E, bm, sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(),
                 expert_offsets.data_ptr<int>(), max_p, total_p.data_ptr<int>(), inv.data_ptr<int>(),
                 cur_stream());
}

void moe_gemm(torch::Tensor X, int64_t topk, torch::Tensor sorted_ids, torch::Tensor tile_expert,
              torch::Tensor W, torch::Tensor Y, int64_t mode, int64_t act, double alpha, double limit,
              bool a_rows_are_slots, c10::optional<torch::Tensor> bias, int64_t tile_m) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(X));
  CHECK_CUDA(X); CHECK_BF16(X); CHECK_BF16(W); CHECK_BF16(Y); CHECK_INNER(X); CHECK_INNER(Y);
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous(), "W [E, N, K] contiguous");
  const int N = W.size(1), K = W.size(2);
  TORCH_CHECK(X.size(1) == K && K % 8 == 0, "moe_gemm: K");
  const bool v3 = tile_m == llmd_moe_gemm3_tile_m();
  TORCH_CHECK(tile_m == 0 || tile_m == llmd_moe_gemm_tile_m() || v3, "moe_gemm: tile_m");
  const int bm = v3 ? llmd_moe_gemm3_tile_m() : llmd_moe_gemm_tile_m();
  const int P = sorted_ids.numel();
  TORCH_CHECK(P % bm == 0 && tile_expert.numel() >= P / bm && Y.size(0) >= P, "moe_gemm: rows");
  TORCH_CHECK(Y.size(1) >= (mode == 1 ? N / 2 : N) && N % 2 == 0, "moe_gemm: Y width");
  TORCH_CHECK(X.stride(0) % 8 == 0, "16-B aligned rows");
  const void* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(bias.value());
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == (int64_t)W.size(0) * N, "bias [E, N]");
    bp = bias->data_ptr();
  }
  if (v3) {
    TORCH_CHECK(K % 32 == 0, "moe_gemm v3: K % 32");
    const int rc = llmd_moe_gemm3_bf16(X.data_ptr(), X.stride(0), topk, sorted_ids.data_ptr<int>(),
                                       tile_expert.data_ptr<int>(), P / bm, W.data_ptr(), W.stride(0), N, K,
                                       Y.data_ptr(), Y.stride(0), mode, act, (float)alpha, (float)limit,
                                       a_rows_are_slots ? 1 : 0, bp, cur_stream());
    TORCH_CHECK(rc == 0, "moe_gemm v3 failed: ", rc);
    return;
  }
  llmd_moe_gemm(X.data_ptr(), X.stride(0), topk, sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(), P / bm,
                W.data_ptr(), W.stride(0), N, K, Y.data_ptr(), Y.stride(0), mode, act, (float)alpha, (float)limit,
                a_rows_are_slots ? 1 : 0, bp, cur_stream());
}

// bf16 grouped GEMM v4 (csrc/ops/moe4.hip) on the 256-row expert tiles of moe_align(bm = 256)
void moe_gemm4(torch::Tensor X, int64_t topk, torch::Tensor sorted_ids, torch::Tensor tile_expert, torch::Tensor W,
               torch::Tensor Y, int64_t mode, int64_t act, double alpha, double limit, bool a_rows_are_slots,
               c10::optional<torch::Tensor> bias, int64_t tile_m, int64_t version, c10::optional<torch::Tensor> total) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(X));
  TORCH_CHECK(version == 4 || (version == 8 && total.has_value()),
              "moe_gemm4: version 4 (moe4.hip) or 8 (moe8.hip, needs moe_align's total)");
  CHECK_CUDA(X); CHECK_BF16(X); CHECK_BF16(W); CHECK_BF16(Y); CHECK_INNER(X); CHECK_INNER(Y);
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous(), "W [E, N, K] contiguous");
  const int N = W.size(1), K = W.size(2);
  TORCH_CHECK(X.size(1) == K && K % 64 == 0, "moe_gemm4: K % 64");
  TORCH_CHECK(tile_m == 256 || tile_m == 192, "moe_gemm4: tile_m 256 or 192");
  const int bm = (int)tile_m;
  const int P = sorted_ids.numel();
  TORCH_CHECK(P % bm == 0 && tile_expert.numel() >= P / bm && Y.size(0) >= P, "moe_gemm4: rows");
  TORCH_CHECK(Y.size(1) >= (mode == 1 ? N / 2 : N), "moe_gemm4: Y width");
  TORCH_CHECK(X.stride(0) % 8 == 0 && Y.stride(0) % 8 == 0, "16-B aligned rows");
  const void* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(bias.value());
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == (int64_t)W.size(0) * N, "bias [E, N]");
    bp = bias->data_ptr();
  }
  int rc;
  if (version == 8) {
    CHECK_CUDA(total.value()); CHECK_DT(total.value(), at::kInt);
    rc = llmd_moe_gemm8_bf16(X.data_ptr(), X.stride(0), topk, sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(),
                             total->data_ptr<int>(), P / bm, W.data_ptr(), W.stride(0), N, K, Y.data_ptr(),
                             Y.stride(0), mode, act, (float)alpha, (float)limit, a_rows_are_slots ? 1 : 0, bp,
                             X.size(0), bm, cur_stream());
  } else {
    rc = llmd_moe_gemm4_bf16(X.data_ptr(), X.stride(0), topk, sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(),
                             P / bm, W.data_ptr(), W.stride(0), N, K, Y.data_ptr(), Y.stride(0), mode, act,
                             (float)alpha, (float)limit, a_rows_are_slots ? 1 : 0, bp, X.size(0), bm, cur_stream());
  }
  TORCH_CHECK(rc == 0, "moe_gemm4 failed: ", rc);
}

// block-fp8 grouped GEMM v4 (csrc/ops/moe4.hip) or v8 (csrc/ops/moe8.hip, version = 8) on 256 / 192-row expert
// tiles: power-of-two scales, K % 128 == 0
void moe_gemm4_fp8(torch::Tensor X, torch::Tensor xs, int64_t topk, torch::Tensor sorted_ids,
                   torch::Tensor tile_expert, torch::Tensor W, torch::Tensor ws, torch::Tensor Y, int64_t mode,
                   int64_t act, double alpha, double limit, bool a_rows_are_slots, c10::optional<torch::Tensor> bias,
                   int64_t tile_m, int64_t version, c10::optional<torch::Tensor> total) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(X));
  TORCH_CHECK(version == 4 || (version == 8 && total.has_value()),
              "moe_gemm4_fp8: version 4 (moe4.hip) or 8 (moe8.hip, needs moe_align's total)");
  CHECK_CUDA(X); CHECK_DT(X, at::kFloat8_e4m3fn); CHECK_DT(W, at::kFloat8_e4m3fn); CHECK_BF16(Y);
  CHECK_INNER(X); CHECK_INNER(Y); CHECK_DT(xs, at::kFloat); CHECK_DT(ws, at::kFloat);
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous() && ws.is_contiguous(), "W [E, N, K] / ws contiguous");
  const int E = W.size(0), N = W.size(1), K = W.size(2);
  TORCH_CHECK(X.size(1) == K && K % 128 == 0 && K / 128 <= 64 && X.stride(0) % 16 == 0, "moe_gemm4_fp8: K");
  TORCH_CHECK(tile_m == 256 || tile_m == 192 || (tile_m == 64 && version == 8),
              "moe_gemm4_fp8: tile_m 256 or 192 (64: version 8 only)");
  TORCH_CHECK(ws.dim() == 3 && ws.size(0) == E && ws.size(1) == (N + 127) / 128 && ws.size(2) == K / 128,
              "ws [E, ceil(N/128), K/128]");
  TORCH_CHECK(xs.dim() == 2 && xs.size(0) >= X.size(0) && xs.size(1) >= K / 128 && xs.stride(1) == 1,
              "xs [rows, K/128]");
  const int bm = (int)tile_m;
  const int P = sorted_ids.numel();
  TORCH_CHECK(P % bm == 0 && tile_expert.numel() >= P / bm && Y.size(0) >= P, "moe_gemm4_fp8: rows");
  TORCH_CHECK(Y.size(1) >= (mode == 1 ? N / 2 : N) && Y.stride(0) % 8 == 0, "moe_gemm4_fp8: Y width");
  const void* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(bias.value());
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == (int64_t)E * N, "bias [E, N]");
    bp = bias->data_ptr();
  }
  int rc;
  if (version == 8) {
    CHECK_CUDA(total.value()); CHECK_DT(total.value(), at::kInt);
    rc = llmd_moe_gemm8_fp8(X.data_ptr(), X.stride(0), xs.data_ptr<float>(), xs.stride(0), topk,
                            sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(), total->data_ptr<int>(), P / bm,
                            W.data_ptr(), W.stride(0), ws.data_ptr<float>(), N, K, Y.data_ptr(), Y.stride(0), mode,
                            act, (float)alpha, (float)limit, a_rows_are_slots ? 1 : 0, bp, X.size(0), bm,
                            cur_stream());
  } else {
    rc = llmd_moe_gemm4_fp8(X.data_ptr(), X.stride(0), xs.data_ptr<float>(), xs.stride(0), topk,
                            sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(), P / bm, W.data_ptr(),
                            W.stride(0), ws.data_ptr<float>(), N, K, Y.data_ptr(), Y.stride(0), mode, act,
                            (float)alpha, (float)limit, a_rows_are_slots ? 1 : 0, bp, X.size(0), bm, cur_stream());
  }
  TORCH_CHECK(rc == 0, "moe_gemm4_fp8 failed: ", rc);
}

extern "C" int llmd_moe_gemm8_mxfp4(const void*, int64_t, const float*, int64_t, int, const int*, const int*,
                                    const int*, int, const void*, int64_t, const void*, int64_t, int, int, void*,
                                    int64_t, int, int, float, float, int, const void*, int64_t, int, int,
                                    hipStream_t);

// MXFP4 experts on the persistent tile GEMM (csrc/ops/moe8.hip): W [E, N, K/2] packed e2m1, wsc [E, N, K/32]
// E8M0, X [rows, K] e4m3 with power-of-two (token, 128) scales xs
void moe_gemm8_mxfp4(torch::Tensor X, torch::Tensor xs, int64_t topk, torch::Tensor sorted_ids,
                     torch::Tensor tile_expert, torch::Tensor W, torch::Tensor wsc, torch::Tensor Y, int64_t mode,
                     int64_t act, double alpha, double limit, bool a_rows_are_slots,
                     c10::optional<torch::Tensor> bias, int64_t tile_m, torch::Tensor total) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(X));
  CHECK_CUDA(X); CHECK_DT(X, at::kFloat8_e4m3fn); CHECK_DT(W, at::kByte); CHECK_DT(wsc, at::kByte); CHECK_BF16(Y);
  CHECK_INNER(X); CHECK_INNER(Y); CHECK_DT(xs, at::kFloat); CHECK_DT(total, at::kInt);
  // W [E, N, K/2] (the packed standard order) or [E, K/128, N, 64] (K-step major, ops.mxfp4_kernel_layout)
  // K-step major: W [E, K/128, N, 64] with wsc [E, K/128, N, 4] (ops.mxfp4_kernel_layout / _scales_)
  TORCH_CHECK((W.dim() == 3 || (W.dim() == 4 && W.size(3) == 64)) && W.is_contiguous() &&
              wsc.dim() == W.dim() && wsc.is_contiguous(),
              "W [E, N, K/2] + wsc [E, N, K/32], or W [E, K/128, N, 64] + wsc [E, K/128, N, 4], contiguous");
  const bool kmajor = W.dim() == 4;
  const int E = W.size(0), N = kmajor ? W.size(2) : W.size(1), K = kmajor ? 128 * W.size(1) : 2 * W.size(2);
  if (kmajor) {
    TORCH_CHECK(wsc.size(0) == E && wsc.size(1) == K / 128 && wsc.size(2) == N && wsc.size(3) == 4,
                "wsc [E, K/128, N, 4]");
  } else {
    TORCH_CHECK(wsc.size(0) == E && wsc.size(1) == N && wsc.size(2) == K / 32, "wsc [E, N, K/32]");
  }
  TORCH_CHECK(X.size(1) == K && K % 128 == 0 && K / 128 >= 4 && X.stride(0) % 16 == 0, "moe_gemm8_mxfp4: K");
  TORCH_CHECK(tile_m == 256 || tile_m == 192 || tile_m == 64, "moe_gemm8_mxfp4: tile_m 256, 192 or 64");
  TORCH_CHECK(xs.dim() == 2 && xs.size(0) >= X.size(0) && xs.size(1) >= K / 128 && xs.stride(1) == 1, "xs [rows, K/128]");
  const int bm = (int)tile_m;
  const int P = sorted_ids.numel();
  TORCH_CHECK(P % bm == 0 && tile_expert.numel() >= P / bm && Y.size(0) >= P, "moe_gemm8_mxfp4: rows");
  TORCH_CHECK(Y.size(1) >= (mode == 1 ? N / 2 : N) && Y.stride(0) % 8 == 0, "moe_gemm8_mxfp4: Y width");
  const void* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(bias.value());
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == (int64_t)E * N, "bias [E, N]");
    bp = bias->data_ptr();
  }
  const int rc = llmd_moe_gemm8_mxfp4(X.data_ptr(), X.stride(0), xs.data_ptr<float>(), xs.stride(0), topk,
                                      sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(), total.data_ptr<int>(),
                                      P / bm, W.data_ptr(), W.stride(0), wsc.data_ptr(), wsc.stride(0), N, K,
                                      Y.data_ptr(), Y.stride(0), mode, act, (float)alpha, (float)limit,
                                      a_rows_are_slots ? 1 : 0, bp, X.size(0), bm, kmajor ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "moe_gemm8_mxfp4 failed: ", rc);
}

void moe_combine(torch::Tensor Y, torch::Tensor inv, torch::Tensor w, int64_t topk, torch::Tensor out) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(Y));
  CHECK_CUDA(Y); CHECK_BF16(Y); CHECK_BF16(out); CHECK_DT(inv, at::kInt); CHECK_DT(w, at::kFloat);
  const int T = out.size(0), d = out.size(1);
  TORCH_CHECK(d % 8 == 0 && Y.size(1) >= d && inv.numel() >= (int64_t)T * topk && w.numel() >= (int64_t)T * topk,
              "moe_combine shapes");
  llmd_moe_combine(Y.data_ptr(), Y.stride(0), inv.data_ptr<int>(), w.data_ptr<float>(), T, topk, d,
                   out.data_ptr(), out.stride(0), cur_stream());
}

// ---------------------------------------------------------------- fp8 quant
void quant_fp8_rows(torch::Tensor x, torch::Tensor q, torch::Tensor scale) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_INNER(x); CHECK_INNER(q); CHECK_DT(q, at::kFloat8_e4m3fn);
  CHECK_DT(scale, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && q.sizes() == x.sizes() && scale.numel() >= x.size(0), "quant_fp8_rows shapes");
  TORCH_CHECK(x.size(1) % 8 == 0 && x.stride(0) % 8 == 0 && q.stride(0) % 8 == 0, "quant_fp8_rows: 16-B rows");
  int rc = llmd_quant_fp8_rows(x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0), scale.data_ptr<float>(),
                               x.size(0), x.size(1), cur_stream());
  TORCH_CHECK(rc == 0, "quant_fp8_rows failed: ", rc);
}

// q, scale <- fp8(rmsnorm(x [+= residual]) * w)
void rms_norm_quant(torch::Tensor q, torch::Tensor scale, torch::Tensor x, c10::optional<torch::Tensor> residual,
                    torch::Tensor w, double eps) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_INNER(x); CHECK_INNER(q);
  CHECK_DT(q, at::kFloat8_e4m3fn); CHECK_DT(scale, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && q.sizes() == x.sizes() && scale.numel() >= x.size(0), "rms_norm_quant shapes");
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && w.numel() == d && w.is_contiguous(), "rms_norm_quant d");
  TORCH_CHECK(x.stride(0) % 8 == 0 && q.stride(0) % 8 == 0, "16-B aligned rows");
  void* rp = nullptr;
  int64_t rs = 0;
  if (residual.has_value()) {
    CHECK_BF16(residual.value()); CHECK_INNER(residual.value());
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->stride(0) % 8 == 0, "residual shape");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  llmd_rms_norm_quant(q.data_ptr(), q.stride(0), scale.data_ptr<float>(), x.data_ptr(), x.stride(0), rp, rs,
                      w.data_ptr(), x.size(0), d, (float)eps, cur_stream());
}

void gated_act_quant(torch::Tensor q, torch::Tensor scale, torch::Tensor x, int64_t mode, double alpha,
                     double limit) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_INNER(x); CHECK_INNER(q);
  CHECK_DT(q, at::kFloat8_e4m3fn); CHECK_DT(scale, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && q.dim() == 2 && q.size(0) == x.size(0), "gated_act_quant shape");
  const int F = q.size(1);
  TORCH_CHECK(x.size(1) == 2 * F && F % 8 == 0 && scale.numel() >= x.size(0), "gated_act_quant widths");
  TORCH_CHECK(x.stride(0) % 8 == 0 && q.stride(0) % 8 == 0, "16-B aligned rows");
  llmd_gated_act_quant(q.data_ptr(), q.stride(0), scale.data_ptr<float>(), x.data_ptr(), x.stride(0), x.size(0), F,
                       (int)mode, (float)alpha, (float)limit, cur_stream());
}

void quant_fp8_groups(torch::Tensor x, torch::Tensor q, torch::Tensor scale) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_INNER(x); CHECK_INNER(q); CHECK_DT(q, at::kFloat8_e4m3fn);
  CHECK_DT(scale, at::kFloat);
  const int d = x.size(1);
  TORCH_CHECK(x.dim() == 2 && q.sizes() == x.sizes() && d % 8 == 0, "quant_fp8_groups shapes");
  TORCH_CHECK(scale.dim() == 2 && scale.size(0) >= x.size(0) && scale.size(1) >= (d + 127) / 128 &&
                  scale.stride(1) == 1, "quant_fp8_groups: scale [T, ceil(d/128)]");
  TORCH_CHECK(x.stride(0) % 8 == 0 && q.stride(0) % 8 == 0, "16-B rows");
  int rc = llmd_quant_fp8_groups(x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0), scale.data_ptr<float>(),
                                 scale.stride(0), x.size(0), d, cur_stream());
  TORCH_CHECK(rc == 0, "quant_fp8_groups failed: ", rc);
}

// x [T, d] bf16 -> q [T, kp] e4m3 (zeros past d) + per-128 scales; rows >= row_limit[0] skipped when given
void quant_fp8_groups_padded(torch::Tensor x, torch::Tensor q, torch::Tensor scale, c10::optional<torch::Tensor> row_limit) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_INNER(x); CHECK_INNER(q); CHECK_DT(q, at::kFloat8_e4m3fn);
  CHECK_DT(scale, at::kFloat);
  const int d = x.size(1), kp = q.size(1);
  TORCH_CHECK(x.dim() == 2 && q.dim() == 2 && q.size(0) == x.size(0) && d % 8 == 0 && kp % 8 == 0 && kp >= d,
              "quant_fp8_groups_padded shapes");
  TORCH_CHECK(scale.dim() == 2 && scale.size(0) >= x.size(0) && scale.size(1) >= (d + 127) / 128 &&
                  scale.stride(1) == 1, "quant_fp8_groups_padded: scale [T, ceil(d/128)]");
  TORCH_CHECK(x.stride(0) % 8 == 0 && q.stride(0) % 8 == 0, "16-B rows");
  const int* lim = nullptr;
  if (row_limit.has_value()) {
    CHECK_DT((*row_limit), at::kInt);
    lim = row_limit->data_ptr<int>();
  }
  int rc = llmd_quant_fp8_groups_padded(x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0),
                                        scale.data_ptr<float>(), scale.stride(0), x.size(0), d, kp, lim,
                                        cur_stream());
  TORCH_CHECK(rc == 0, "quant_fp8_groups_padded failed: ", rc);
}

void moe_gemm_fp8(torch::Tensor X, torch::Tensor xs, int64_t topk, torch::Tensor sorted_ids, torch::Tensor tile_expert,
                  torch::Tensor W, torch::Tensor ws, torch::Tensor Y, int64_t mode, int64_t act, double alpha,
                  double limit, bool a_rows_are_slots, c10::optional<torch::Tensor> bias, int64_t tile_m,
                  c10::optional<torch::Tensor> hq, c10::optional<torch::Tensor> hs) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(X));
  CHECK_CUDA(X); CHECK_DT(X, at::kFloat8_e4m3fn); CHECK_DT(W, at::kFloat8_e4m3fn); CHECK_BF16(Y);
  CHECK_INNER(X); CHECK_INNER(Y); CHECK_DT(xs, at::kFloat); CHECK_DT(ws, at::kFloat);
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous() && ws.is_contiguous(), "W [E, N, K] / ws contiguous");
  const int E = W.size(0), N = W.size(1), K = W.size(2);
  TORCH_CHECK(X.size(1) == K && K % 16 == 0 && X.stride(0) % 16 == 0, "moe_gemm_fp8: K");
  TORCH_CHECK(ws.dim() == 3 && ws.size(0) == E && ws.size(1) == (N + 127) / 128 && ws.size(2) == (K + 127) / 128,
              "ws [E, ceil(N/128), ceil(K/128)]");
  TORCH_CHECK(xs.dim() == 2 && xs.size(0) >= X.size(0) && xs.size(1) >= (K + 127) / 128 && xs.stride(1) == 1,
              "xs [rows, ceil(K/128)]");
  const bool v3 = tile_m == llmd_moe_gemm3_tile_m();
  TORCH_CHECK(tile_m <= 0 || tile_m == llmd_moe_gemm_tile_m() || v3, "moe_gemm_fp8: tile_m");
  const int bm = v3 ? (int)tile_m : llmd_moe_gemm_tile_m();
  const int P = sorted_ids.numel();
  const bool fused = hq.has_value();  // the output is hq / hs; Y is unused
  TORCH_CHECK(P % bm == 0 && tile_expert.numel() >= P / bm && (fused || Y.size(0) >= P), "moe_gemm_fp8: rows");
  TORCH_CHECK((fused || Y.size(1) >= (mode == 1 ? N / 2 : N)) && N % 2 == 0, "moe_gemm_fp8: Y width");
  const void* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16(bias.value());
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == (int64_t)E * N, "bias [E, N]");
    bp = bias->data_ptr();
  }
  void* hqp = nullptr;
  float* hsp = nullptr;
  int64_t hq_stride = 0, hs_stride = 0;
  if (hq.has_value()) {  // fused activation quantisation (256-row tiles, mode 1)
    TORCH_CHECK(v3 && mode == 1 && hs.has_value(), "fused quant: 256-row tiles, gated activation, hq + hs");
    CHECK_DT(hq.value(), at::kFloat8_e4m3fn); CHECK_INNER(hq.value()); CHECK_DT(hs.value(), at::kFloat);
    TORCH_CHECK(hq->size(0) >= P && hq->size(1) >= ((N / 2 + 127) / 128) * 128 && hq->size(1) % 128 == 0,
                "hq [rows, F rounded up to 128]");
    TORCH_CHECK(hs->dim() == 2 && hs->size(0) >= P && hs->size(1) >= (N + 255) / 256 && hs->stride(1) == 1,
                "hs [rows, F / 128]");
    hqp = hq->data_ptr();
    hsp = hs->data_ptr<float>();
    hq_stride = hq->stride(0);
    hs_stride = hs->stride(0);
  }
  if (v3) {  // 256-row expert tiles: power-of-two scales, K % 128 == 0, 16-B rows
    TORCH_CHECK(K % 128 == 0 && X.stride(0) % 16 == 0 && W.stride(0) % 16 == 0, "moe_gemm_fp8 (256-row tiles): K");
    const int rc = llmd_moe_gemm3_fp8(X.data_ptr(), X.stride(0), xs.data_ptr<float>(), xs.stride(0), topk,
                                      sorted_ids.data_ptr<int>(), tile_expert.data_ptr<int>(), P / bm, W.data_ptr(),
                                      W.stride(0), ws.data_ptr<float>(), N, K, fused ? nullptr : Y.data_ptr(),
                                      fused ? 0 : Y.stride(0), mode, act, (float)alpha, (float)limit,
                                      a_rows_are_slots ? 1 : 0, bp, hqp, hq_stride, hsp, hs_stride, cur_stream());
    TORCH_CHECK(rc == 0, "moe_gemm3_fp8 failed: ", rc);
    return;
  }
  llmd_moe_gemm_fp8(X.data_ptr(), X.stride(0), xs.data_ptr<float>(), xs.stride(0), topk, sorted_ids.data_ptr<int>(),
                    tile_expert.data_ptr<int>(), P / bm, W.data_ptr(), W.stride(0), ws.data_ptr<float>(), N, K,
                    Y.data_ptr(), Y.stride(0), mode, act, (float)alpha, (float)limit, a_rows_are_slots ? 1 : 0, bp,
                    cur_stream());
}

// ---------------------------------------------------------------- symm heap
torch::Tensor symm_alloc(int64_t bytes, int64_t device) {
  const c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  TORCH_CHECK(bytes > llmd_symm_sig_bytes() && bytes % 4096 == 0, "symm_alloc: size");
  void* p = nullptr;
  int rc = llmd_symm_alloc((size_t)bytes, &p);
  TORCH_CHECK(rc == 0, "symm_alloc (hipExtMallocWithFlags uncached) failed: ", rc);
  return torch::from_blob(p, {bytes}, [](void* q) { llmd_symm_free(q); },
                          torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, (c10::DeviceIndex)device));
}

int64_t symm_error(torch::Tensor heap, bool clear) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(heap));
  uint32_t e = 0;
  TORCH_CHECK(llmd_symm_error(heap.data_ptr(), &e) == 0, "symm_error: copy failed");
  if (clear) llmd_symm_clear_error(heap.data_ptr());
  return (int64_t)e;
}

// address of the process's host-mapped symm failure word (allocated on first use)
int64_t symm_host_err() {
  int64_t p = 0;
  TORCH_CHECK(llmd_symm_host_err(&p) == 0, "symm_host_err: hipHostMalloc failed");
  return p;
}

void check_bases(const std::vector<int64_t>& bases, int64_t rank) {
  TORCH_CHECK((int)bases.size() >= 1 && (int)bases.size() <= llmd_symm_max_ranks(), "symm: 1..8 ranks");
  TORCH_CHECK(rank >= 0 && rank < (int64_t)bases.size(), "symm: rank");
  for (auto b : bases) TORCH_CHECK(b != 0 && b % 256 == 0, "symm: bad peer base");
}

void symm_all_reduce(std::vector<int64_t> bases, int64_t rank, int64_t ch, int64_t mode, int64_t data_off,
                     int64_t slot_bytes, torch::Tensor inp, torch::Tensor out) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(inp));
  check_bases(bases, rank);
  CHECK_CUDA(inp); CHECK_BF16(inp); CHECK_BF16(out);
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.numel() == out.numel(), "all_reduce: contiguous");
  TORCH_CHECK(inp.numel() % 8 == 0, "all_reduce: numel % 8");
  TORCH_CHECK(data_off >= llmd_symm_sig_bytes() && (mode == 1 || mode == 2), "all_reduce: layout/mode");
  int rc = llmd_symm_all_reduce(bases.data(), (int)bases.size(), (int)rank, (int)ch, (int)mode, data_off, slot_bytes,
                                inp.data_ptr(), out.data_ptr(), inp.numel() / 8, cur_stream());
  TORCH_CHECK(rc == 0, "symm_all_reduce failed: ", rc);
}

void symm_ep_dispatch(std::vector<int64_t> bases, int64_t rank, int64_t ch, std::vector<int64_t> layout,
                      torch::Tensor x, torch::Tensor ids, torch::Tensor w, int64_t R, int64_t E_local, bool fp8) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(x));
  check_bases(bases, rank);
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_INNER(x); CHECK_DT(ids, at::kInt); CHECK_DT(w, at::kFloat);
  TORCH_CHECK(layout.size() == 7, "ep layout");
  TORCH_CHECK(!fp8 || (layout[5] >= 0 && layout[6] >= 0), "ep_dispatch: heap has no fp8 receive area");
  const int T = x.size(0), d = x.size(1);
  TORCH_CHECK(ids.dim() == 2 && ids.is_contiguous() && w.sizes() == ids.sizes() && w.is_contiguous() &&
                  ids.size(0) == T, "ep_dispatch: ids/w [T, k]");
  const int k = ids.size(1);
  TORCH_CHECK(T <= R && d % 8 == 0 && k <= 64 && x.stride(0) % 8 == 0, "ep_dispatch shape");
  int rc = llmd_symm_ep_dispatch(bases.data(), (int)bases.size(), (int)rank, (int)ch, layout.data(), x.data_ptr(),
                                 x.stride(0), ids.data_ptr<int>(), w.data_ptr<float>(), T, (int)R, d, k, (int)E_local,
                                 (int)fp8, cur_stream());
  TORCH_CHECK(rc == 0, "symm_ep_dispatch failed: ", rc);
}

void symm_ep_combine(std::vector<int64_t> bases, int64_t rank, int64_t ch, std::vector<int64_t> layout,
                     torch::Tensor y, torch::Tensor ids, int64_t R, int64_t E_local, torch::Tensor out) {
  const c10::hip::OptionalHIPGuard device_guard(dev_of(y));
  check_bases(bases, rank);
  CHECK_CUDA(y); CHECK_BF16(y); CHECK_BF16(out); CHECK_INNER(y); CHECK_INNER(out); CHECK_DT(ids, at::kInt);
  TORCH_CHECK(layout.size() == 7, "ep layout");
  const int T = out.size(0), d = out.size(1);
  TORCH_CHECK(ids.dim() == 2 && ids.is_contiguous() && ids.size(0) == T, "ep_combine: ids [T, k]");
  TORCH_CHECK(y.size(0) == (int64_t)bases.size() * R && y.size(1) >= d && d % 8 == 0 && T <= R, "ep_combine shape");
  TORCH_CHECK(y.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "16-B aligned rows");
  int rc = llmd_symm_ep_combine(bases.data(), (int)bases.size(), (int)rank, (int)ch, layout.data(), y.data_ptr(),
                                y.stride(0), ids.data_ptr<int>(), T, (int)R, d, (int)ids.size(1), (int)E_local,
                                out.data_ptr(), out.stride(0), cur_stream());
  TORCH_CHECK(rc == 0, "symm_ep_combine failed: ", rc);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {  // _C, or _C_debug (llmd_amd/build.py)
  m.doc() = "llmd_amd HIP/CDNA4 op library (gfx950)";
  m.def("rms_norm", &rms_norm);
  m.def("fused_add_rms_norm", &fused_add_rms_norm);
  m.def("qk_rms_norm", &qk_rms_norm, "Qwen3 per-head q/k RMSNorm in place in the fused QKV output");
  m.def("layer_norm", &layer_norm);
  m.def("rope_cache", &rope_cache);
  m.def("gated_act", &gated_act);
  m.def("paged_decode", &paged_decode);
  m.def("paged_prefill", &paged_prefill);
  m.def("kv_dequant_gather", &kv_dequant_gather);
  m.def("moe_gemm8_mxfp4", &moe_gemm8_mxfp4);
  m.def("prefill_tokens_per_item", [](int64_t Hq, int64_t Hkv, int64_t D, int64_t bs, bool fp8) {
    return llmd_prefill_tokens_per_item((int)Hq, (int)Hkv, (int)D, (int)bs, fp8 ? 1 : 0);
  });
  m.def("sample", &sample);
  m.def("topk_topp_mask", &topk_topp_mask);
  m.def("kvx_copy_blocks", &kvx_copy_blocks);
  m.def("kvx_dma_blocks", &kvx_dma_blocks);
  m.def("kvx_ipc_export", &kvx_ipc_export);
  m.def("kvx_ipc_open", &kvx_ipc_open);
  m.def("kvx_ipc_close", &kvx_ipc_close);
  m.def("mla_attention", &mla_attention);
  m.def("mla_v2_shape", &mla_v2_shape, "H=128 MLA kernel shape: 10 * waves + head blocks per wave");
  m.def("skinny_gemm", &skinny_gemm);
  m.def("skinny_supported", &skinny_supported);
  m.def("mgemm", &mgemm);
  m.def("mgemm_partials", &mgemm_partials, "split-K partials of the medium-M GEMM (no reduce); returns nsplit");
  m.def("reduce_rope_cache", &reduce_rope_cache, "QKV split-K reduce + RoPE + paged cache write");
  m.def("mgemm_add_rmsnorm", &mgemm_add_rmsnorm, "decode o / down projection with residual-add + RMSNorm in its split-K reduce");
  m.def("pgemm_fp8", &pgemm_fp8, "prefill fp8 W8A8 GEMM (256x256 LDS-DMA tiles on 16x16x128 f8f6f4 MFMA), "
        "per-token x per-channel scales, optional fused SiLU-and-mul");
  m.def("pgemm", &pgemm, "prefill bf16 GEMM (256x256 LDS-DMA MFMA tiles), optional fused SiLU-and-mul",
        py::arg("y"), py::arg("x"), py::arg("w"), py::arg("epi"), py::arg("variant"), py::arg("split_k") = true);
  m.def("mgemm_fp8", &mgemm_fp8);
  m.def("mgemm_lds", [](int64_t M, int64_t wrb, int64_t stages) { return llmd_mgemm_lds((int)M, (int)wrb, (int)stages); });
  m.def("lora_bgmv", &lora_bgmv);
  m.def("mla_rope_cache", &mla_rope_cache);
  m.def("vmm_granularity", &vmm_granularity);
  m.def("vmm_pool", &vmm_pool);
  m.def("vmm_import", &vmm_import);
  m.def("vmm_release", &vmm_release);
  m.def("moe_topk", &moe_topk);
  m.def("moe_align", &moe_align, py::arg("ids"), py::arg("E"), py::arg("sorted_ids"), py::arg("tile_expert"),
        py::arg("expert_offsets"), py::arg("total_p"), py::arg("inv"), py::arg("tile_m") = 0);
  m.def("moe_gemm", &moe_gemm, py::arg("X"), py::arg("topk"), py::arg("sorted_ids"), py::arg("tile_expert"),
        py::arg("W"), py::arg("Y"), py::arg("mode"), py::arg("act"), py::arg("alpha"), py::arg("limit"),
        py::arg("a_rows_are_slots"), py::arg("bias"), py::arg("tile_m") = 0);
  m.def("moe_combine", &moe_combine);
  m.def("moe_tile_m", &llmd_moe_gemm_tile_m);
  m.def("quant_fp8_rows", &quant_fp8_rows);
  m.def("quant_fp8_groups", &quant_fp8_groups);
  m.def("quant_fp8_groups_padded", &quant_fp8_groups_padded, py::arg("x"), py::arg("q"), py::arg("scale"),
        py::arg("row_limit") = py::none());
  m.def("rms_norm_quant", &rms_norm_quant);
  m.def("gated_act_quant", &gated_act_quant);
  m.def("moe_gemm_fp8", &moe_gemm_fp8, py::arg("X"), py::arg("xs"), py::arg("topk"), py::arg("sorted_ids"),
        py::arg("tile_expert"), py::arg("W"), py::arg("ws"), py::arg("Y"), py::arg("mode"), py::arg("act"),
        py::arg("alpha"), py::arg("limit"), py::arg("a_rows_are_slots"), py::arg("bias"), py::arg("tile_m") = 0,
        py::arg("hq") = py::none(), py::arg("hs") = py::none());
  m.def("moe_tile_m_prefill", &llmd_moe_gemm3_tile_m);
  m.def("symm_alloc", &symm_alloc);
  m.def("moe_gemm4", &moe_gemm4, py::arg("X"), py::arg("topk"), py::arg("sorted_ids"), py::arg("tile_expert"),
        py::arg("W"), py::arg("Y"), py::arg("mode"), py::arg("act"), py::arg("alpha"), py::arg("limit"),
        py::arg("a_rows_are_slots"), py::arg("bias"), py::arg("tile_m") = 256, py::arg("version") = 4,
        py::arg("total") = py::none());
  m.def("mgemm_silu", &mgemm_silu);
  m.def("moe_gemm4_fp8", &moe_gemm4_fp8, py::arg("X"), py::arg("xs"), py::arg("topk"), py::arg("sorted_ids"),
        py::arg("tile_expert"), py::arg("W"), py::arg("ws"), py::arg("Y"), py::arg("mode"), py::arg("act"),
        py::arg("alpha"), py::arg("limit"), py::arg("a_rows_are_slots"), py::arg("bias"), py::arg("tile_m") = 256,
        py::arg("version") = 4, py::arg("total") = py::none());
  m.def("symm_error", &symm_error);
  m.def("symm_host_err", &symm_host_err);
  m.def("symm_sig_bytes", &llmd_symm_sig_bytes);
  m.def("symm_grid", &llmd_symm_grid);
  m.def("symm_channels", &llmd_symm_channels);
  m.def("symm_all_reduce", &symm_all_reduce);
  m.def("symm_ep_dispatch", &symm_ep_dispatch, py::arg("bases"), py::arg("rank"), py::arg("ch"), py::arg("layout"),
        py::arg("x"), py::arg("ids"), py::arg("w"), py::arg("R"), py::arg("E_local"), py::arg("fp8") = false);
  m.def("symm_ep_combine", &symm_ep_combine);
}
