"""GPU busy fraction from a rocprofv3 kernel trace CSV over the last `window`
seconds of the run: union of kernel intervals / wall span.
  python scripts/busy_from_trace.py <kernel_trace.csv> [window_s]"""
import csv
import sys


def main():
    path = sys.argv[1]
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    iv = []
    with open(path) as f:
        for row in csv.DictReader(f):
            iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row.get("Kernel_Name", "")))
    iv.sort()
    end = max(e for _, e, _ in iv)
    lo = end - int(window * 1e9)
    sel = [(max(s, lo), e, n) for s, e, n in iv if e > lo]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = end - lo
    gaps = []
    prev = None
    for s, e, n in sel:
        if prev is not None and s - prev > 200_000:
            gaps.append((s - prev) / 1e6)
        prev = max(prev or 0, e)
    print(f"window {window:.1f}s: GPU busy {busy / span * 100:.1f}% ({busy / 1e9:.3f}s of {span / 1e9:.3f}s); "
          f"kernels {len(sel)}; idle gaps >0.2ms: {len(gaps)} totalling {sum(gaps):.1f} ms, "
          f"largest {max(gaps) if gaps else 0:.1f} ms")


def breakdown(path, window):
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row.get("Kernel_Name", "")))
    end = max(e for _, e, _ in rows)
    lo = end - int(window * 1e9)
    agg = {}
    for s, e, n in rows:
        if e > lo:
            k = n.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0][:90] or "<unnamed>"
            t, c = agg.get(k, (0, 0))
            agg[k] = (t + e - max(s, lo), c + 1)
    tot = sum(t for t, _ in agg.values())
    print(f"per-kernel time in the last {window:.1f}s (total kernel {tot / 1e6:.1f} ms):")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:24]:
        print(f"  {t / 1e6:9.1f} ms {100 * t / tot:5.1f}% {c:6d}  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "--breakdown":
        breakdown(sys.argv[1], float(sys.argv[2]))
    main()
