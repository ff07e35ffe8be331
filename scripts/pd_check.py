"""P/D correctness across processes and devices: one
prefill engine (rank 0, TP1) hands requests to a decode replica (ranks 1 ..
dtp, TP ``--decode-tp``) through the kvx connector, and the decoder's greedy
tokens must equal an aggregated engine's on the same weights (a first
divergence is allowed only as a near-tie of the reference, tests/greedy_check.py,
when the decoder's TP layout sums in another order).

Launched with torch.distributed.run (1 + dtp ranks, --master-addr 127.0.0.1).
``LLMD_PD_DEVICES`` maps ranks to devices ("0,0": the 1-GPU rehearsal, P and D
share cuda:0 and still pull through IPC-mapped memory; "0,1": across xGMI).
Distinct devices run the world over RCCL, which the ``rccl`` transport and a
TP2 decoder need; shared devices use gloo (ipc transport, TP1 only).

  --model small-llama | tiny-gpt-oss (hybrid KV: the windowed pool moves too)
  --transport ipc | rccl ; LLMD_KV_VMM=0 exports a plain hipMalloc pool instead
  of the VMM-chunked one.
Prints ``PDCHECK {json}`` on rank 0 and exits non-zero on any mismatch.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="small-llama")
    ap.add_argument("--transport", default="ipc")
    ap.add_argument("--decode-tp", type=int, default=1)
    ap.add_argument("--max-tokens", type=int, default=12)
    ap.add_argument("--lens", default="143,150,77,300")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu",
                    help="cpu: the harness itself over gloo + the tcp transport (CI rehearsal)")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dtp = a.decode_tp
    assert world == 1 + dtp, (world, dtp)
    devs = [int(x) for x in os.environ.get("LLMD_PD_DEVICES", ",".join(str(r) for r in range(world))).split(",")]
    dev = devs[rank]
    gpu = a.device == "cuda"
    if gpu:
        torch.cuda.set_device(dev)
    distinct = gpu and len(set(devs)) == len(devs)
    to = datetime.timedelta(seconds=300)
    if distinct:
        dist.init_process_group("nccl", rank=rank, world_size=world, timeout=to,
                                device_id=torch.device("cuda", dev))
    else:
        assert dtp == 1 and a.transport in ("ipc", "tcp"), "shared devices: ipc / tcp transport, TP1 decoder only"
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=to)
    allg = dist.new_group(backend="gloo", timeout=to)           # start-up barrier (every rank)
    ctl = dist.new_group([0, 1], backend="gloo", timeout=to)    # prefill <-> decode driver exchange
    is_follower = False
    if dtp > 1:
        from llmd_amd.parallel.state import ParallelState, set_state

        ranks = list(range(1, world))
        tg = dist.new_group(ranks, timeout=to)
        tgc = dist.new_group(ranks, backend="gloo", timeout=to)
        if rank in ranks:
            set_state(ParallelState(world_size=world, rank=rank, local_rank=dev, tp_size=dtp, tp_rank=rank - 1,
                                    tp_group=tg, tp_cpu_group=tgc, cpu_group=tgc, backend=dist.get_backend(),
                                    tp_src=1))
            is_follower = rank != 1
    if a.transport == "rccl":
        from llmd_amd.kvx.agent import set_p2p_group

        set_p2p_group(dist.new_group(timeout=to))

    from llmd_amd.engine.config import EngineConfig
    from llmd_amd.engine.engine import LLMEngine
    from llmd_amd.engine.request import SamplingParams

    is_prefill = rank == 0
    os.environ.setdefault("LLMD_PD_BASE_PORT", str(18600 + 10 * (os.getpid() % 500)))
    kt = {"kv_connector": "KvxConnector", "kv_role": "kv_producer" if is_prefill else "kv_consumer",
          "kv_connector_extra_config": {"transport": a.transport, "require_ipc": a.transport == "ipc"}}
    common = dict(device=a.device, block_size=16, num_gpu_blocks=256, max_num_batched_tokens=512, max_num_seqs=8,
                  max_model_len=1024, seed=0)
    cfg = EngineConfig.create(a.model, kv_transfer_config=kt, tensor_parallel_size=dtp if not is_prefill else 1,
                              **common)
    lens = [int(x) for x in a.lens.split(",")]
    rng = np.random.default_rng(7)
    prompts = [rng.integers(3, 500, size=n).tolist() for n in lens]
    sp = SamplingParams(max_tokens=a.max_tokens, temperature=0.0, ignore_eos=True)

    if is_follower:
        from llmd_amd.engine.tp_worker import run_follower

        run_follower(cfg, on_ready=lambda: dist.barrier(group=allg))
        sys.exit(0)  # released by the driver's shutdown; rank 0 decides the result

    eng = LLMEngine(cfg)
    dist.barrier(group=allg)  # every engine (and its kvx server) is up
    res = {"model": a.model, "transport": a.transport, "decode_tp": dtp, "devices": devs,
           "vmm": os.environ.get("LLMD_KV_VMM", "1")}
    if is_prefill:
        ktps = []
        for i, p in enumerate(prompts):
            eng.add_request(f"p{i}", p, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True),
                            kv_transfer_params={"do_remote_decode": True})
            ktps.append(None)
        t = time.monotonic() + 120
        while any(k is None for k in ktps) and time.monotonic() < t:
            for o in eng.step():
                if o.finished:
                    ktps[int(o.request_id[1:])] = o.kv_transfer_params
        objs = [ktps]
        dist.broadcast_object_list(objs, src=0, group=ctl)
        # serve the decoder's pulls (agent threads) and release held blocks on engine ticks
        got = [None]
        done = {"v": False}
        import threading

        def recv():
            dist.broadcast_object_list(got, src=1, group=ctl)
            done["v"] = True
        th = threading.Thread(target=recv, daemon=True)
        th.start()
        while not done["v"]:
            eng.step()
            time.sleep(0.002)
        th.join()
        # reference: an aggregated TP1 engine on the same weights
        ref = LLMEngine(EngineConfig.create(a.model, **common))
        want = [r.output_token_ids for r in ref.generate(prompts, sp)]
        from greedy_check import first_divergences

        div = first_divergences(ref, prompts, got[0]["tokens"], want)
        bad = [d for d in div if not d["near_tie"]]
        res.update({"exact": sum(1 for g, w in zip(got[0]["tokens"], want) if g == w), "n": len(prompts),
                    "divergences": div, "decoder": got[0]["stats"]})
        ok = bool(got[0]["stats"]["all_remote"]) and not bad
        res["ok"] = ok
        print("PDCHECK " + json.dumps(res), flush=True)
        dist.broadcast_object_list([ok], src=0, group=ctl)
        sys.exit(0 if ok else 1)
    else:
        objs = [None]
        dist.broadcast_object_list(objs, src=0, group=ctl)
        ktps = objs[0]
        reqs = [eng.add_request(f"d{i}", p, sp, kv_transfer_params=k) for i, (p, k) in enumerate(zip(prompts, ktps))]
        t = time.monotonic() + 180
        while eng.has_unfinished() and time.monotonic() < t:
            eng.step()
            if eng.last_step_empty:
                time.sleep(0.002)
        stats = {"all_remote": all(r.num_cached_tokens == len(p) - 1 for r, p in zip(reqs, prompts)),
                 "cached": [r.num_cached_tokens for r in reqs], "finished": not eng.has_unfinished()}
        dist.broadcast_object_list([{"tokens": [r.output_token_ids for r in reqs], "stats": stats}], src=1, group=ctl)
        ok = [None]
        dist.broadcast_object_list(ok, src=0, group=ctl)
        eng.shutdown()
        sys.exit(0 if ok[0] else 1)


if __name__ == "__main__":
    main()
