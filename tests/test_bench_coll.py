"""scripts/bench_coll.py (RCCL collective / xGMI point-to-point bandwidth
microbenchmark) runs its full op list over gloo with 2 ranks on the CPU and
emits one well-formed JSON row per (op, size)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_coll_gloo_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29577", os.path.join(ROOT, "scripts", "bench_coll.py"),
           "--device", "cpu", "--min-bytes", "4096", "--max-bytes", "65536", "--iters", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    ops = {row["op"] for row in rows}
    assert ops == {"all_reduce", "all_gather", "reduce_scatter", "all_to_all", "sendrecv"}
    assert len(rows) == 5 * 3 and all(row["ranks"] == 2 and row["us"] > 0 for row in rows)
    ar = [row for row in rows if row["op"] == "all_reduce"][0]
    assert abs(ar["busbw_GBs"] - ar["algbw_GBs"]) < 0.02 + 1e-6 * ar["algbw_GBs"]  # 2(n-1)/n = 1 at n = 2
