"""Scan a hipcc --save-temps .s file for two hazards of MFMAs issued from inline asm, which
hipcc does not model: accumulator reads that follow an asm MFMA writing the same AGPRs too
closely (register-allocator copies in its shadow), and VALU writes of a VGPR that an asm MFMA
issued shortly before still reads as SrcA / SrcB (the allocator reuses an operand register
right after its last asm use - moe4.hip's 192-row form computed wrong rows from it). Prints each
suspect and the counts.
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
    # WAR: a VALU write of a VGPR that an asm MFMA issued shortly before still reads as SrcA / SrcB
    func, war, in_asm = None, 0, False
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l):
            func = l.split(":")[0]
        if ";;#ASMSTART" in l:
            in_asm = True
        elif ";;#ASMEND" in l:
            in_asm = False
        m = re.search(r"v_mfma\S*\s+a\[\d+:\d+\],\s*v\[(\d+):(\d+)\],\s*v\[(\d+):(\d+)\]", l)
        if not m or not in_asm:
            continue
        srcs = set(range(int(m.group(1)), int(m.group(2)) + 1)) | set(range(int(m.group(3)), int(m.group(4)) + 1))
        n = 0
        for l2 in lines[i + 1:i + 60]:
            t = l2.strip()
            if not t or t.startswith(";") or t.endswith(":") or t.startswith("."):
                continue
            n += int(t.split()[1]) + 1 if t.startswith("s_nop") else 1
            if n >= need:
                break
            w = re.match(r"(v_(?!mfma|accvgpr_read)\S+)\s+v\[?(\d+)(?::(\d+))?\]?", t)
            if w:
                lo = int(w.group(2))
                hi = int(w.group(3)) if w.group(3) else lo
                if srcs & set(range(lo, hi + 1)):
                    print(f"{func[:90]}: line {i + 1}: WAR {t} {n} states after {l.strip()[:60]}")
                    war += 1
                    break
    print(f"{path}: {bad} accumulator suspects, {war} operand WAR suspects")


if __name__ == "__main__":
    main()
