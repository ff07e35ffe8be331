"""Probe the chunked VMM pool export/import (kvx_vmm.hip) between two
processes on one GPU: exporter builds an N-GiB pool of 2-GiB chunks, passes the
dmabuf fds over a Unix socket (SCM_RIGHTS), importer maps and copies from it.
Usage: python scripts/vmm_probe.py GB"""
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CHUNK = 2 << 30


def exporter(gb, path):
    from llmd_amd import _C

    n = max(1, int(gb * (1 << 30)) // CHUNK)
    t0 = time.time()
    pool, fds = _C.vmm_pool(0, CHUNK, n)
    pool.view(torch.bfloat16)[:: (1 << 20)].fill_(3.0)
    pool.view(torch.bfloat16)[-8:].fill_(5.0)
    torch.cuda.synchronize()
    print(f"[exp] pool {n} x 2 GiB in {time.time() - t0:.2f}s", flush=True)
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(1)
    c, _ = srv.accept()
    socket.send_fds(c, [len(fds).to_bytes(4, "little")], fds)
    c.recv(1)  # importer done
    print("[exp] done", flush=True)


def importer(gb, path):
    from llmd_amd import _C

    while not os.path.exists(path):
        time.sleep(0.05)
    c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    c.connect(path)
    msg, fds, _, _ = socket.recv_fds(c, 16, 1024)
    t0 = time.time()
    base = _C.vmm_import(list(fds), CHUNK, 0)
    print(f"[imp] import {len(fds)} chunks in {time.time() - t0:.3f}s", flush=True)
    total = len(fds) * CHUNK
    dst = torch.zeros(8, dtype=torch.bfloat16, device="cuda")
    pairs = torch.tensor([[0, 0]], dtype=torch.int32, device="cuda")
    seg = torch.tensor([[total - 16, 0, 16]], dtype=torch.int64, device="cuda")
    _C.kvx_copy_blocks(dst, base, 16, 0, pairs, seg, 16, 1)
    torch.cuda.synchronize()
    print(f"[imp] tail copy ok={bool((dst == 5.0).all())}", flush=True)
    _C.vmm_release(base)
    c.send(b"x")


if __name__ == "__main__":
    if len(sys.argv) > 3:
        role, gb, path = sys.argv[1], float(sys.argv[2]), sys.argv[3]
        exporter(gb, path) if role == "exp" else importer(gb, path)
        sys.exit(0)
    gb = sys.argv[1]
    path = f"/tmp/vmm_probe_{os.getpid()}.sock"
    pe = subprocess.Popen([sys.executable, __file__, "exp", gb, path])
    pi = subprocess.Popen([sys.executable, __file__, "imp", gb, path])
    rc = pi.wait(timeout=120)
    pe.wait(timeout=30)
    sys.exit(rc or pe.returncode)
