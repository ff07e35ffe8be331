"""Merge TunableOp result CSVs into the committed table (later files win per key).
Validator lines come from the first file; every file must agree on them.
  python scripts/merge_tunableop.py llmd_amd/tuning/tunableop_gfx950.csv new1.csv [new2.csv ...]
(the first file is rewritten in place)"""
import sys


def read(path):
    val, rows = {}, {}
    with open(path) as f:
        for line in f:
            parts = line.rstrip("\n").split(",")
            if len(parts) < 3:
                continue
            if parts[0] == "Validator":
                val[parts[1]] = parts[2]
            else:
                rows[(parts[0], parts[1])] = line.rstrip("\n")
    return val, rows


def main():
    dst, srcs = sys.argv[1], sys.argv[2:]
    val, rows = read(dst)
    for s in srcs:
        v, r = read(s)
        for k in ("PT_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION", "GCN_ARCH_NAME"):
            if k in v and k in val and v[k] != val[k]:
                raise SystemExit(f"{s}: validator {k}={v[k]} != {val[k]}")
        rows.update(r)
    with open(dst, "w") as f:
        for k, v in val.items():
            f.write(f"Validator,{k},{v}\n")
        for line in rows.values():
            f.write(line + "\n")
    print(f"{dst}: {len(rows)} entries")


if __name__ == "__main__":
    main()
