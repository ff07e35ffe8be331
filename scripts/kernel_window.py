"""Per-kernel time over the last `window` seconds of a rocprofv3 kernel trace (the timed window of
a bench run ends the trace): total ms, share and count per kernel name, plus the GPU busy share.
  python scripts/kernel_window.py <kernel_trace.csv | results.db> [window_s] [top]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    iv = []
    if path.endswith(".db"):  # rocprofv3's default rocpd SQLite output
        import sqlite3

        con = sqlite3.connect(path)
        iv = [(int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels")]
    else:
        with open(path) as f:
            for row in csv.DictReader(f):
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row.get("Kernel_Name", "")))
    end = max(e for _, e, _ in iv)
    lo = end - int(window * 1e9)
    tot, cnt = defaultdict(int), defaultdict(int)
    sel = sorted((max(s, lo), e, n) for s, e, n in iv if e > lo)
    for s, e, n in sel:
        tot[n] += e - s
        cnt[n] += 1
    busy, cs, ce = 0, None, None
    for s, e, _ in sel:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
    allk = sum(tot.values())
    print(f"per-kernel time in the last {window:.1f}s (total kernel {allk / 1e6:.1f} ms, GPU busy "
          f"{100 * busy / (end - lo):.1f} %):")
    for n, t in sorted(tot.items(), key=lambda x: -x[1])[:top]:
        print(f"  {t / 1e6:9.1f} ms {100 * t / allk:5.1f}% {cnt[n]:6d}  {n[:110]}")


if __name__ == "__main__":
    main()
