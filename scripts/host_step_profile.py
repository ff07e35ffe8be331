"""Host time of a decode step outside the forward: scheduler, block tables,
plan (_prepare), sampling bookkeeping, update. Tiny model on the CPU, 64 running
sequences at ~1k context (the bench's decode batch), cProfile over 30 steps.
  python scripts/host_step_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmd_amd.engine.config import EngineConfig  # noqa: E402
from llmd_amd.engine.engine import LLMEngine  # noqa: E402
from llmd_amd.engine.request import SamplingParams  # noqa: E402

B, CTX = int(os.environ.get("B", 64)), int(os.environ.get("CTX", 1024))
cfg = EngineConfig.create("tiny-llama", device="cpu", block_size=64, num_gpu_blocks=B * (CTX // 64 + 4) + 8,
                          max_num_batched_tokens=8192, max_num_seqs=B, max_model_len=CTX + 256,
                          enforce_eager=True)
eng = LLMEngine(cfg)
rng = np.random.default_rng(0)
for i in range(B):
    eng.add_request(f"r{i}", rng.integers(3, 400, size=CTX).tolist(),
                    SamplingParams(max_tokens=200, temperature=0.0, ignore_eos=True))
while eng.sched.waiting or any(r.num_computed_tokens < r.num_prompt_tokens for r in eng.sched.running):
    eng.step()
for _ in range(3):
    eng.step()
fw = [0.0]
orig = eng.runner.run_plan


def timed(pl):
    t = time.perf_counter()
    r = orig(pl)
    fw[0] += time.perf_counter() - t
    return r


eng.runner.run_plan = timed
N = 30
t0 = time.perf_counter()
for _ in range(N):
    eng.step()
tot = time.perf_counter() - t0
print(f"B={B} ctx={CTX}: step {tot / N * 1e3:.3f} ms, forward {fw[0] / N * 1e3:.3f} ms, "
      f"host outside forward {(tot - fw[0]) / N * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    eng.step()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(
    r"engine\.py:\d+\(step\)|schedule|block_table|plan\b|_prepare|_sample|update|_finish_step|on_step|"
    r"_sampling_tensors|_sample_rows|_flush_events|check_health")
