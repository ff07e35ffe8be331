"""A/B of the two kvx block-copy engines (csrc/ops/kvx_copy.hip) on the layouts
the P/D pull and the offload tier actually move:

* engine 0: register-staged (4 x 16-B loads in flight per lane, non-temporal stores);
* engine 1: LDS-staged (global_load_lds 16 KB per wave into LDS, then stores).

Cases, on a Llama-3-70B layer-major bf16 pool [80 layers, NB blocks, K/V, 8 heads,
block, 128] (the engine's ``runner.kv`` layout):
* ``pull``     - pool -> pool, one segment per layer (a TP-matched P/D pull);
* ``reslice``  - pool -> pool, TP1 -> TP2 head slice: one segment per (layer,
  K/V plane) of 4 of the 8 heads (a TP2 decoder pulling its half);
* ``pack``     - pool -> block-major staging slab (the offload tier's D2H pack);
* ``unpack``   - slab -> pool (the reload scatter).
Block sizes 64 and 128 tokens; transfers of 1, 16, 79 and 128 blocks with random
source blocks. Every case is checked against a torch gather of the same bytes,
then both engines are timed in interleaved rounds in one process. Same-device
memory: the kernels' own rate; a cross-GPU pull adds the xGMI link.

  python bench/kvx_copy_ab.py [--rounds 5] [--blocks 64,128]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--blocks", default="64,128")
    ap.add_argument("--nb", type=int, default=160, help="blocks per pool")
    a = ap.parse_args()
    from llmd_amd import _C

    dev = torch.device("cuda", 0)
    L, H, D = 80, 8, 128
    torch.manual_seed(0)
    for bs in (int(b) for b in a.blocks.split(",")):
        NB = a.nb
        src = torch.randint(-30000, 30000, (L, NB, 2, H, bs, D), dtype=torch.int16, device=dev).view(torch.bfloat16)
        dst = torch.zeros_like(src)
        esz = 2
        lbb = 2 * H * bs * D * esz            # one block of one layer
        lstride = NB * lbb                    # layer stride of the layer-major pool
        head = bs * D * esz
        blk = L * lbb                         # one block, all layers
        print(f"block {bs} tokens: {blk / 2**20:.1f} MiB per block ({lbb // 1024} KiB per layer)", flush=True)
        dst2 = torch.zeros(L, NB, 2, H // 2, bs, D, dtype=torch.bfloat16, device=dev)  # a TP2 decoder's pool
        lbb2, lstride2 = lbb // 2, NB * lbb // 2
        cases = {
            "pull": [(l * lstride, l * lstride, lbb) for l in range(L)],
            "reslice": [(l * lstride + (p * H + 0) * head, l * lstride2 + p * (H // 2) * head, (H // 2) * head)
                        for l in range(L) for p in range(2)],
            "pack": [(l * lstride, l * lbb, lbb) for l in range(L)],
        }
        for nblk in (1, 16, 79, 128):
            sids = torch.randperm(NB)[:nblk]
            dids = torch.randperm(NB)[:nblk]
            stage = torch.empty(nblk, blk, dtype=torch.uint8, device=dev)
            for name in ("pull", "reslice", "pack", "unpack"):
                if name == "unpack":
                    segs = [(l * lbb, l * lstride, lbb) for l in range(L)]
                    s_ptr, s_stride, d_t, d_stride = stage.data_ptr(), blk, dst, lbb
                    pairs = torch.stack([torch.arange(nblk), dids], 1)
                elif name == "pack":
                    segs = cases[name]
                    s_ptr, s_stride, d_t, d_stride = src.data_ptr(), lbb, stage, blk
                    pairs = torch.stack([sids, torch.arange(nblk)], 1)
                elif name == "reslice":
                    segs = cases[name]
                    s_ptr, s_stride, d_t, d_stride = src.data_ptr(), lbb, dst2, lbb2
                    pairs = torch.stack([sids, dids], 1)
                else:
                    segs = cases[name]
                    s_ptr, s_stride, d_t, d_stride = src.data_ptr(), lbb, dst, lbb
                    pairs = torch.stack([sids, dids], 1)
                pr = pairs.int().to(dev)
                sg = torch.tensor(segs, dtype=torch.int64, device=dev)
                mx = max(x[2] for x in segs)
                nbytes = nblk * sum(x[2] for x in segs)

                def run(engine):
                    _C.kvx_copy_blocks(d_t, s_ptr, d_stride, s_stride, pr, sg, mx, engine)

                # correctness of both engines against a torch gather of the same bytes
                ok = {}
                for eng in (0, 1):
                    d_t.zero_()
                    if name == "unpack":
                        stage.copy_(src[:, sids].transpose(0, 1).reshape(nblk, -1).view(torch.uint8))
                    run(eng)
                    torch.cuda.synchronize()
                    # compare bit patterns (int16 views): random bf16 bits include NaNs, and NaN != NaN
                    if name == "pull":
                        ok[eng] = bool(torch.equal(dst[:, dids].view(torch.int16), src[:, sids].view(torch.int16)))
                    elif name == "reslice":
                        ok[eng] = bool(torch.equal(dst2[:, dids].view(torch.int16),
                                                   src[:, sids, :, : H // 2].view(torch.int16)))
                    elif name == "pack":
                        want = src[:, sids].transpose(0, 1).reshape(nblk, -1).view(torch.uint8)
                        ok[eng] = bool(torch.equal(stage, want))
                    else:
                        ok[eng] = bool(torch.equal(dst[:, dids].view(torch.int16), src[:, sids].view(torch.int16)))
                ts = {0: [], 1: []}
                for _ in range(a.rounds):
                    for eng in (0, 1):
                        ts[eng].append(timeit(lambda: run(eng)))
                med = {e: sorted(v)[len(v) // 2] for e, v in ts.items()}
                print(f"  {name:8s} {nblk:4d} blocks ({nbytes / 2**20:8.1f} MiB, {len(segs)} segs/block): "
                      f"reg {med[0] * 1e3:8.1f} us {nbytes / med[0] / 1e6:7.1f} GB/s | "
                      f"lds {med[1] * 1e3:8.1f} us {nbytes / med[1] / 1e6:7.1f} GB/s | lds/reg "
                      f"{med[0] / med[1]:.3f} | ok reg={ok[0]} lds={ok[1]}", flush=True)
            del stage
        del src, dst, dst2


if __name__ == "__main__":
    main()
