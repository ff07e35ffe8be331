"""xGMI peer-copy bandwidth matrix (SURVEY N19 rdma-tools role, single node):
for every (src, dst) GPU pair, time a 1 GiB device-to-device copy (SDMA
engines over xGMI); the diagonal is the local HBM copy rate.
  python bench/xgmi_bw.py [--mb 1024]"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024)
    a = ap.parse_args()
    n = torch.cuda.device_count()
    nbytes = a.mb << 20
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{i}") for i in range(n)]
    print("GB/s  " + " ".join(f"dst{j:<5d}" for j in range(n)))
    for i in range(n):
        row = []
        for j in range(n):
            src, dst = bufs[i], (bufs[j] if i != j else torch.empty_like(bufs[j]))
            dst.copy_(src)
            torch.cuda.synchronize(j)
            t0 = time.perf_counter()
            for _ in range(5):
                dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize(i)
            torch.cuda.synchronize(j)
            row.append(5 * nbytes / (time.perf_counter() - t0) / 1e9)
        print(f"src{i:<2d} " + " ".join(f"{v:8.1f}" for v in row), flush=True)


if __name__ == "__main__":
    main()
