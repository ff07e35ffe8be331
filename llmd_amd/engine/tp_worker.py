"""Tensor-parallel follower ranks (SURVEY §2.5 TP, M01/M02).

One process per GPU. TP rank 0 of a replica runs the full engine (scheduler,
block manager, API); every other TP rank runs only a ModelRunner holding its
weight and KV-head shard. Each step the driver broadcasts the step plan
(token ids, positions, slots, block tables, sequence lengths, sample rows;
``ModelRunner.plan``) over the replica's gloo group and all ranks execute the
same forward - RCCL all-reduces inside the layers keep them in lock-step, and
decode buckets replay the same hipGraphs on every rank. Logits are
all-gathered by the LM head; only the driver samples.

Start-up mirrors the driver exactly (profile -> agree on the block count with
a MIN all-reduce -> allocate -> capture graphs), so collectives line up.
"""
from __future__ import annotations

import logging

import torch

from llmd_amd.parallel import symm as _symm
from llmd_amd.parallel.comm import tp_broadcast_plan, tp_recv_plan

from .config import EngineConfig
from .model_runner import ModelRunner

log = logging.getLogger("llmd.tp")

STOP = {"stop": True}


def run_follower(cfg: EngineConfig, capture_graphs: bool = True, on_ready=None) -> int:
    """Blocking loop for TP ranks != 0. Returns the number of steps executed.
    ``on_ready`` runs once the runner is built (the driver's engine is up at
    the same point), before the first plan is received."""
    runner = ModelRunner(cfg)
    runner.profile_and_allocate()
    if cfg.enable_lora:
        from .engine import make_lora_manager

        make_lora_manager(cfg, runner, driver=False)
    kvx = None
    if cfg.kv_transfer_config:
        from llmd_amd.kvx.connector import KvxFollower

        kvx = KvxFollower(cfg, runner)
    if capture_graphs:
        runner.capture_graphs()
    if on_ready is not None:
        on_ready()
    n = 0
    with torch.no_grad():
        while True:
            pl = tp_recv_plan()
            if pl is None or pl.get("stop"):
                break
            if "lora_cmd" in pl:  # adapter load/unload issued on the driver
                runner.lora.apply_cmd(pl["lora_cmd"])
                continue
            if "ws_cmd" in pl:  # RL weight sync / sleep / wake issued on the driver
                if getattr(runner, "weight_sync", None) is None:
                    from .weight_sync import WeightSync

                    runner.weight_sync = WeightSync(runner)
                try:  # a failed update (bad path, ...) fails on the driver too: stay in the loop
                    runner.weight_sync.apply(pl["ws_cmd"])
                except Exception:  # noqa: BLE001
                    log.exception("weight-sync command %s failed", pl["ws_cmd"].get("op"))
                continue
            if "kvx_cmd" in pl:  # P/D: KV pulls / cancels scheduled on the driver
                kvx.apply(pl)
                continue
            runner.run_plan(pl)
            _symm.check_health("follower plan %d" % n)  # a stalled peer: exit non-zero, never continue
            n += 1
    if kvx is not None:
        kvx.close()
    log.info("tp follower exiting after %d steps", n)
    return n


def stop_followers():
    """Driver side: release the followers' loops."""
    tp_broadcast_plan(STOP)
