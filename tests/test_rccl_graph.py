"""RCCL collectives inside a hipGraph capture (GPU only). The TP decode
replicas of the P/D bench replay captured decode graphs whose LM head
all-gathers logits with RCCL (parallel/comm.py tp_all_gather) after the
communicator was created outside the capture (comm.warm_tp_group). One GPU
cannot host two RCCL ranks, so this pins the capture mechanics - communicator
warm-up, capture, replay on fresh inputs - on a one-rank group."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_all_gather_and_all_reduce_replay_in_graph():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from llmd_amd.parallel.comm import warm_tp_group
        from llmd_amd.parallel.state import ParallelState, get_state, set_state

        g = dist.new_group([0])
        prev = get_state()
        set_state(ParallelState(world_size=1, rank=0, tp_size=2, tp_group=g, backend="nccl"))
        try:
            # tp_size=2 state over a one-rank group: warm_tp_group issues both collectives
            warm_tp_group(torch.device("cuda", 0))
        finally:
            set_state(prev)
        x = torch.randn(64, 1000, device="cuda")
        y = torch.empty(64, 1000, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # one eager round on the capture stream first
            dist.all_gather_into_tensor(y, x * 2, group=g)
            z = x.clone()
            dist.all_reduce(z, group=g)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            dist.all_gather_into_tensor(y, x * 2, group=g)
            z = x.clone()
            dist.all_reduce(z, group=g)
        for _ in range(3):
            x.copy_(torch.randn_like(x))
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(y, x * 2) and torch.equal(z, x)
    finally:
        dist.destroy_process_group()
