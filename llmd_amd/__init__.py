"""llmd_amd: an MI355X-native (gfx950 / CDNA4) distributed LLM inference serving stack.

Layers (bottom-up, see docs/ARCHITECTURE.md):
  ops/       hand-written HIP kernels (MFMA paged attention, fused norms, rope+cache, sampling)
  models/    Llama / Qwen3 / gpt-oss (MoE) on the paged-KV engine
  parallel/  torch.distributed over RCCL/xGMI: TP, DP, EP collectives, custom all-reduce
  engine/    continuous-batching engine: scheduler, native block manager (APC), model runner
  serving/   OpenAI-compatible HTTP server, Prometheus metrics, KV events
  kvx/       P/D KV transfer (NIXL-equivalent) over xGMI / RCCL / TCP
  kvcache/   precise prefix index, tiered KV offload (host DRAM, filesystem)
  router/    EPP: plugin scheduler, flow control, data layer, proxy
  sidecar/   P/D routing sidecar
  batch/     OpenAI Batch API gateway and async processor
  autoscale/ saturation / WVA-style autoscaling signals
  sim/       GPU-free engine simulator
"""
__version__ = "0.1.0"
