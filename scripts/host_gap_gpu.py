"""Where the host time between decode graph replays goes, on the real bench
(bench.py's engine, setup and step loop; sections timed by wrapping the engine's
methods). GPU-busy window per step ~ [run_plan start, _sample end] (the step
syncs on the sampled ids); everything else in the step is host time with the GPU
idle.  python scripts/host_gap_gpu.py --steps 20 --warmup 5"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from llmd_amd.engine import engine as E  # noqa: E402
from llmd_amd.engine import metrics as M  # noqa: E402
from llmd_amd.engine import model_runner as R  # noqa: E402
from llmd_amd.engine import scheduler as S  # noqa: E402

cur = collections.defaultdict(float)
rows = []


def wrap(cls, name, key):
    f = getattr(cls, name)

    def w(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            cur[key] += time.perf_counter() - t
    setattr(cls, name, w)


wrap(S.Scheduler, "schedule", "schedule")
wrap(S.Scheduler, "update", "sched_update")
wrap(E.LLMEngine, "block_tables", "block_tables")
wrap(R.ModelRunner, "plan", "plan")
wrap(R.ModelRunner, "run_plan", "run_plan(copies+replay launch)")
wrap(R.ModelRunner, "_sample", "_sample(incl. GPU wait)")
wrap(M.EngineMetrics, "on_step", "metrics.on_step")
wrap(E.LLMEngine, "_finish_step", "_finish_step(total)")
step = E.LLMEngine.step


last_end = [None]


def st(self):
    cur.clear()
    t = time.perf_counter()
    between = t - last_end[0] if last_end[0] is not None else 0.0  # the caller's loop between steps
    out = step(self)
    last_end[0] = time.perf_counter()
    cur["caller between steps"] = between
    rows.append((self.last_num_tokens, last_end[0] - t, dict(cur)))
    return out


E.LLMEngine.step = st
sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
dec = [r for r in rows[-200:] if r[0] == 64]
if dec:
    keys = sorted({k for r in dec for k in r[2]})
    n = len(dec)
    wall = sum(r[1] for r in dec) / n
    print(f"[gap] decode steps: {n}, mean wall {wall * 1e3:.3f} ms", flush=True)
    for k in keys:
        print(f"[gap]   {k:34s} {sum(r[2].get(k, 0) for r in dec) / n * 1e3:8.3f} ms", flush=True)
    busy = sum(r[2].get("run_plan(copies+replay launch)", 0) + r[2].get("_sample(incl. GPU wait)", 0) for r in dec) / n
    print(f"[gap]   host outside run_plan+_sample      {(wall - busy) * 1e3:8.3f} ms", flush=True)
