"""A/B of the GQA prefill attention v2 schedule variants (csrc/ops/attn_prefill.hip template V,
LLMD_PREFILL_V2_VARIANT, read once per process): one child process per (round, variant),
rounds interleaved, Llama-3-70B heads 64/8, D 128, block 64. Numerics of each variant are
checked against the PyTorch reference in its first round.
  python scripts/attn_v2_variants_ab.py [--variants 5,21,37,53] [--rounds 3]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(5000, 5000), (8192, 8192), (8192, 4096), (2048, 2048)]
D64 = os.environ.get("AB_D64") == "1"  # gpt-oss shape: D 64, 64 / 8 heads (full-attention layers)

CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
from scripts.bench_attn import prefill
out = {{}}
for ctx, ql in {cases!r}:
    out[f"{{ctx}}/{{ql}}"] = prefill(ctx, ql, 64, 8, {D}, 64, check={check!r} and ctx == 2048)
print("RESULT " + json.dumps(out), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="5,21,37,53")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    res = {}
    for r in range(a.rounds):
        for v in a.variants.split(","):
            # "v5": the software-pipelined kernel (csrc/ops/attn_prefill5.hip); numbers: v2 variants
            env = dict(os.environ, LLMD_PREFILL_V5="1") if v == "v5" else dict(os.environ, LLMD_PREFILL_V2_VARIANT=v)
            code = CHILD.format(root=ROOT, cases=CASES, check=(r == 0), D=64 if D64 else 128)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
            for k, t in json.loads(line[7:]).items():
                res.setdefault((k, v), []).append(t)
            print(f"round {r} variant {v} done", flush=True)
    for ctx, ql in CASES:
        k = f"{ctx}/{ql}"
        vis = sum(ctx - ql + i + 1 for i in range(ql))
        fl = 4 * 64 * (64 if D64 else 128) * vis
        parts = []
        for v in a.variants.split(","):
            t = sorted(res[(k, v)])[len(res[(k, v)]) // 2]
            parts.append(f"{v if v.startswith('v') else 'V' + v} {t * 1e3:.3f} ms {fl / t / 1e12:.0f} TF/s")
        print(f"AB ctx={ctx} q={ql}: " + " | ".join(parts), flush=True)


if __name__ == "__main__":
    main()
