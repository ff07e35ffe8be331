"""kvx READ benchmark (SURVEY N02 nixlbench role): the decode side pulls KV
blocks from a producer's VMM-chunked pool with the kvx copy kernel, for a range
of blocks-per-transfer, with a consistency check of every pulled block.

  python bench/kvx_bench.py [--src-dev 0 --dst-dev 1] [--block-mb 20] [--pool-gb 16]

One producer and one consumer process (same GPU or two GPUs of one node: the
pull then runs over xGMI). Default block = one Llama-3-70B bf16 KV block of 64
tokens (80 layers x 2 x 8 heads x 64 x 128 x 2 B = 20 MiB)."""
import argparse
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CHUNK = 2 << 30


def producer(a, path):
    from llmd_amd import _C

    torch.cuda.set_device(a.src_dev)
    block = int(a.block_mb * (1 << 20))
    nblocks = int(a.pool_gb * (1 << 30)) // block
    n = (nblocks * block + CHUNK - 1) // CHUNK
    pool, fds = _C.vmm_pool(a.src_dev, CHUNK, n)
    view = pool[: nblocks * block].view(torch.int32).view(nblocks, block // 4)
    view.copy_(torch.arange(nblocks, device=pool.device, dtype=torch.int32)[:, None].expand_as(view))
    torch.cuda.synchronize()
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(1)
    c, _ = srv.accept()
    socket.send_fds(c, [nblocks.to_bytes(4, "little")], fds)
    c.recv(1)


def consumer(a, path):
    from llmd_amd import _C

    torch.cuda.set_device(a.dst_dev)
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > 60:
            raise SystemExit("producer did not come up")
        time.sleep(0.05)
    c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    c.connect(path)
    msg, fds, _, _ = socket.recv_fds(c, 16, 256)
    nblocks = int.from_bytes(msg[:4], "little")
    base = _C.vmm_import(list(fds), CHUNK, a.dst_dev)
    block = int(a.block_mb * (1 << 20))
    dst = torch.empty(128, block // 4, dtype=torch.int32, device=f"cuda:{a.dst_dev}")
    print(f"pool {nblocks} blocks x {block / 2**20:.1f} MiB, src cuda:{a.src_dev} -> dst cuda:{a.dst_dev}")
    for nb in (1, 4, 16, 79, 128):
        src_ids = torch.randperm(nblocks)[:nb]
        pairs = torch.stack([src_ids, torch.arange(nb)], 1).int().to(dst.device)
        segs = torch.tensor([[0, 0, block]], dtype=torch.int64, device=dst.device)
        fn = lambda: _C.kvx_copy_blocks(dst, base, block, block, pairs, segs, block, a.engine)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        ok = bool((dst[:nb] == src_ids.to(dst.device).int()[:, None]).all())
        t0 = time.perf_counter()
        it = 10
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / it
        print(f"  {nb:4d} blocks ({nb * block / 2**20:8.1f} MiB): {t * 1e3:8.3f} ms  "
              f"{nb * block / t / 1e9:7.1f} GB/s  consistent={ok}", flush=True)
    _C.vmm_release(base)
    c.send(b"x")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src-dev", type=int, default=0)
    ap.add_argument("--dst-dev", type=int, default=0)
    ap.add_argument("--block-mb", type=float, default=20.0)
    ap.add_argument("--engine", type=int, default=1, help="1 = LDS-staged copy kernel, 0 = register-staged")
    ap.add_argument("--pool-gb", type=float, default=8.0)
    ap.add_argument("--role", default=None)
    ap.add_argument("--path", default=None)
    a = ap.parse_args()
    if a.role:
        (producer if a.role == "p" else consumer)(a, a.path)
        return
    path = f"/tmp/kvx_bench_{os.getpid()}.sock"
    common = [sys.executable, __file__, "--src-dev", str(a.src_dev), "--dst-dev", str(a.dst_dev), "--block-mb",
              str(a.block_mb), "--pool-gb", str(a.pool_gb), "--path", path]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.Popen(common + ["--role", "p"], env=env)
    c = subprocess.Popen(common + ["--role", "c"], env=env)
    try:
        rc = c.wait(timeout=300)
        p.wait(timeout=60)
    finally:
        for proc in (p, c):
            if proc.poll() is None:
                proc.kill()
    sys.exit(rc or p.returncode)


if __name__ == "__main__":
    main()
