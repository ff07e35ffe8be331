"""AsyncEngine: drives ``LLMEngine.step()`` on a dedicated thread and fans
outputs out to per-request asyncio queues.

The GPU loop never runs on the event loop: HTTP handlers submit commands
(add / abort / pause / resume / reset) through a thread-safe queue, the engine
thread applies them between steps and pushes ``RequestOutput``s back with
``loop.call_soon_threadsafe``. ``drain(timeout)`` implements graceful shutdown
(``--shutdown-timeout`` semantics, SURVEY §5.3 "Graceful drain").
"""
from __future__ import annotations

import asyncio
import logging
import os
import queue
import threading
import time
from typing import AsyncIterator, Optional

import torch

from llmd_amd.engine.engine import LLMEngine
from llmd_amd.engine.request import RequestOutput, SamplingParams
from llmd_amd.parallel.symm import CollectiveFailure

log = logging.getLogger("llmd.async")


class EngineDeadError(RuntimeError):
    pass


class AsyncEngine:
    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self.cmds: "queue.Queue[tuple]" = queue.Queue()
        self.streams: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self.wake = threading.Event()
        self.stop_flag = False
        self.dead: Optional[BaseException] = None
        self.accepting = True
        self.thread = threading.Thread(target=self._loop, name="llmd-engine", daemon=True)
        self.thread.start()

    # ------------------------------------------------------------ engine thread
    def _loop(self):
        eng = self.engine
        dev = getattr(eng.runner, "device", None)
        if dev is not None and torch.device(dev).type == "cuda":
            torch.cuda.set_device(dev)  # the current HIP device is per thread
        try:
            while not self.stop_flag:
                self._apply_cmds()
                # DP-lockstep (wide-EP) ranks step even when idle: busy peers need
                # this rank in every MoE collective
                if (eng.has_unfinished() or getattr(eng, "dp_lockstep", False)) and not eng.paused \
                        and not getattr(eng, "sleeping", 0) and not getattr(eng, "weights_pending", False):
                    outs = eng.step()
                    for o in outs:
                        self._emit(o)
                    if getattr(eng, "dp_lockstep", False) and eng.last_global_idle:
                        time.sleep(0.001)
                    elif eng.last_step_empty:
                        # only remote-KV waits pending: do not spin
                        time.sleep(0.0005)
                    if eng.connector is not None:
                        for o in eng.connector.take_outputs():
                            self._emit(o)
                else:
                    if getattr(eng, "_pending", None) is not None:  # async: the step in flight's outputs
                        for o in eng.drain():
                            self._emit(o)
                    if eng.connector is not None:
                        eng.connector.tick()
                        for o in eng.connector.take_outputs():
                            self._emit(o)
                    self.wake.wait(0.005 if eng.has_unfinished() else 0.05)
                    self.wake.clear()
        except BaseException as e:  # pragma: no cover - surfaced to clients
            log.exception("engine loop died")
            self.dead = e
            for rid, (loop, q) in list(self.streams.items()):
                loop.call_soon_threadsafe(q.put_nowait, e)
            if isinstance(e, CollectiveFailure) and os.environ.get("LLMD_EXIT_ON_COLLECTIVE_FAILURE", "1") == "1":
                # like NCCL's watchdog abort: the peers are wedged in the same collective, so a
                # restart of the whole replica (the pod) is the only recovery; exit non-zero
                # once the failing streams have been told
                time.sleep(0.5)
                log.critical("exiting: %s", e)
                os._exit(70)

    def _apply_cmds(self):
        while True:
            try:
                cmd = self.cmds.get_nowait()
            except queue.Empty:
                return
            op = cmd[0]
            try:
                if op == "add":
                    _, rid, toks, params, prio, ktp, lora, arrival, mm = cmd
                    self.engine.add_request(rid, toks, params, prio, ktp, lora, arrival, mm_inputs=mm)
                elif op == "abort":
                    self.engine.abort(cmd[1])
                    self._close(cmd[1], None)
                elif op == "call":
                    fn, fut, loop = cmd[1], cmd[2], cmd[3]
                    try:
                        res = fn(self.engine)
                        loop.call_soon_threadsafe(fut.set_result, res)
                    except Exception as e:  # noqa: BLE001
                        loop.call_soon_threadsafe(fut.set_exception, e)
            except Exception as e:  # noqa: BLE001
                if op == "add":
                    self._close(cmd[1], e)

    def _emit(self, o: RequestOutput):
        ent = self.streams.get(o.request_id)
        if ent is None:
            return
        loop, q = ent
        loop.call_soon_threadsafe(q.put_nowait, o)
        if o.finished:
            self.streams.pop(o.request_id, None)

    def _close(self, rid, err):
        ent = self.streams.pop(rid, None)
        if ent is not None:
            loop, q = ent
            loop.call_soon_threadsafe(q.put_nowait, err if err is not None else StopAsyncIteration())

    # ------------------------------------------------------------ API (event loop)
    async def generate(self, request_id: str, prompt_token_ids: list[int], params: SamplingParams,
                       priority: int = 0, kv_transfer_params: Optional[dict] = None,
                       lora_id: int = 0, mm_inputs: Optional[list] = None) -> AsyncIterator[RequestOutput]:
        if self.dead is not None:
            raise EngineDeadError(str(self.dead))
        if not self.accepting:
            raise EngineDeadError("server is shutting down")
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        self.streams[request_id] = (loop, q)
        self.cmds.put(("add", request_id, prompt_token_ids, params, priority, kv_transfer_params,
                       lora_id, time.monotonic(), mm_inputs))
        self.wake.set()
        try:
            while True:
                item = await q.get()
                if isinstance(item, StopAsyncIteration):
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item
                if item.finished:
                    return
        finally:
            if request_id in self.streams:
                self.streams.pop(request_id, None)
                self.cmds.put(("abort", request_id))
                self.wake.set()

    def abort(self, request_id: str):
        self.cmds.put(("abort", request_id))
        self.wake.set()

    async def call(self, fn):
        """Run fn(engine) on the engine thread between steps."""
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self.cmds.put(("call", fn, fut, loop))
        self.wake.set()
        return await fut

    def pause(self):
        self.engine.paused = True

    def resume(self):
        self.engine.paused = False
        self.wake.set()

    async def drain(self, timeout: float):
        self.accepting = False
        t0 = time.monotonic()
        while self.streams and time.monotonic() - t0 < timeout:
            await asyncio.sleep(0.05)
        for rid in list(self.streams):
            self.abort(rid)

    def shutdown(self):
        self.stop_flag = True
        self.wake.set()
        self.thread.join(timeout=5)
        if hasattr(self.engine, "shutdown"):
            self.engine.shutdown()
