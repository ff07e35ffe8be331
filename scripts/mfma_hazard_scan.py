"""Scan a hipcc --save-temps .s file for accumulator reads that follow an asm MFMA writing the
same AGPRs too closely (hipcc does not model the latency of MFMAs issued from inline asm, so
register-allocator copies can land inside their shadow). Prints each suspect and a count.
  python scripts/mfma_hazard_scan.py file.s [min_wait_states=20]"""
import re
import sys


def main():
    path = sys.argv[1]
    need = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lines = open(path).read().split("\n")
    func, bad, in_asm = None, 0, False
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l):
            func = l.split(":")[0]
        if ";;#ASMSTART" in l:
            in_asm = True
        elif ";;#ASMEND" in l:
            in_asm = False
        m = re.search(r"v_mfma\S*\s+a\[(\d+):(\d+)\]", l)
        if not m or not in_asm:  # builtin MFMAs: hipcc's hazard recognizer pads them itself
            continue
        lo, hi = int(m.group(1)), int(m.group(2))
        n = 0
        for l2 in lines[i + 1:i + 60]:
            t = l2.strip()
            if not t or t.startswith(";") or t.endswith(":") or t.startswith(".") or t.startswith("s_endpgm"):
                continue
            if "v_mfma" in t:
                break
            n += int(t.split()[1]) + 1 if t.startswith("s_nop") else 1
            if n >= need:
                break
            r = re.search(r"v_accvgpr_(?:read_b32 v\d+|mov_b32 a\d+), a(\d+)", t)
            if r and lo <= int(r.group(1)) <= hi:
                print(f"{func[:90]}: line {i + 1}: {t} {n} states after {l.strip()[:50]}")
                bad += 1
                break
    print(f"{path}: {bad} suspects")


if __name__ == "__main__":
    main()
