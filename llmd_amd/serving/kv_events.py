"""KV-cache events: engine publisher and router-side subscriber.

Semantics follow the reference's KV-event contract (vLLM ``--kv-events-config``
consumed by the llm-d KV indexer, docs/architecture/advanced/kv-management/
kv-indexer.md:57-87): ``BlockStored{block_hashes, parent_block_hash, token_ids,
block_size, lora_id, medium}``, ``BlockRemoved{block_hashes, medium}``,
``AllBlocksCleared``; batches are published under the topic
``kv@<pod-ip>:<port>@<model>``.

Transport: ZMQ is not available in this stack, so PUB/SUB is a small TCP
protocol with the same roles. The publisher binds ``tcp://*:5556``; a
subscriber connects, sends its topic-prefix filter as one frame, then receives
frames ``[u32 len][topic][u32 len][msgpack payload]``. Slow subscribers are
dropped (high-water mark) rather than blocking the engine.
"""
from __future__ import annotations

import asyncio
import logging
import os
import queue
import socket
import struct
import threading
import time
from typing import Callable, Optional

import msgpack

log = logging.getLogger("llmd.kvevents")
HWM = 10000


def encode_batch(events: list, block_size: int, medium0: str = "GPU") -> dict:
    """Engine BlockManager events -> wire dicts."""
    out = []
    for ev in events:
        kind, h, parent, block, tokens = ev[:5]
        medium = ev[5].upper() if len(ev) > 5 else medium0
        if kind == 0:
            out.append({"type": "BlockStored", "block_hashes": [int(h)], "parent_block_hash": int(parent),
                        "token_ids": list(tokens), "block_size": block_size, "lora_id": None, "medium": medium})
        elif kind == 1:
            out.append({"type": "BlockRemoved", "block_hashes": [int(h)], "medium": medium})
        else:
            out.append({"type": "AllBlocksCleared"})
    return {"ts": time.time(), "events": out}


def _frame(b: bytes) -> bytes:
    return struct.pack("<I", len(b)) + b


def parse_endpoint(ep: str) -> tuple[str, int]:
    ep = ep.replace("tcp://", "")
    host, port = ep.rsplit(":", 1)
    return ("0.0.0.0" if host in ("*", "") else host), int(port)


class KVEventPublisher:
    def __init__(self, endpoint: str, topic: str, block_size: int, medium: str = "GPU"):
        self.host, self.port = parse_endpoint(endpoint)
        self.topic = topic
        self.block_size = block_size
        self.medium = medium
        self.subs: list[tuple[socket.socket, bytes, "queue.Queue[bytes]"]] = []
        self.lock = threading.Lock()
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((self.host, self.port))
        self.port = self.sock.getsockname()[1]
        self.sock.listen(64)
        self.closed = False
        self.seq = 0
        threading.Thread(target=self._accept, daemon=True, name="kv-events-accept").start()

    @classmethod
    def from_config(cls, kcfg: dict, model: str, block_size: int) -> "KVEventPublisher":
        ep = kcfg.get("endpoint", "tcp://*:5556")
        topic = kcfg.get("topic") or f"kv@{os.environ.get('POD_IP', '127.0.0.1')}:" \
                                      f"{os.environ.get('POD_PORT', '8000')}@{model}"
        topic = os.path.expandvars(topic.replace("$(", "${").replace(")", "}"))
        return cls(ep, topic, block_size)

    def _accept(self):
        while not self.closed:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            try:
                c.settimeout(5.0)
                n = struct.unpack("<I", _recvn(c, 4))[0]
                filt = _recvn(c, n)
                c.settimeout(None)
            except (OSError, struct.error):
                c.close()
                continue
            q: "queue.Queue[bytes]" = queue.Queue(maxsize=HWM)
            with self.lock:
                self.subs.append((c, filt, q))
            threading.Thread(target=self._writer, args=(c, q), daemon=True).start()

    def _writer(self, c, q):
        while not self.closed:
            b = q.get()
            if b is None:
                break
            try:
                c.sendall(b)
            except OSError:
                break
        with self.lock:
            self.subs = [s for s in self.subs if s[0] is not c]
        c.close()

    def publish(self, events: list):
        """Called by the engine with BlockManager.take_events() tuples."""
        if not events:
            return
        self.publish_batch(encode_batch(events, self.block_size, self.medium))

    def publish_batch(self, batch: dict, topic: Optional[str] = None):
        t = (topic or self.topic).encode()
        self.seq += 1
        batch = dict(batch, seq=self.seq)
        msg = _frame(t) + _frame(msgpack.packb(batch, use_bin_type=True))
        with self.lock:
            subs = list(self.subs)
        for c, filt, q in subs:
            if t.startswith(filt):
                try:
                    q.put_nowait(msg)
                except queue.Full:  # drop slow subscriber
                    q.put(None)

    def close(self):
        self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass
        with self.lock:
            for _, _, q in self.subs:
                try:
                    q.put_nowait(None)
                except queue.Full:
                    pass


def _recvn(c: socket.socket, n: int) -> bytes:
    buf = b""
    while len(buf) < n:
        chunk = c.recv(n - len(buf))
        if not chunk:
            raise OSError("closed")
        buf += chunk
    return buf


class KVEventSubscriber:
    """asyncio subscriber: connects to a publisher and calls
    ``on_batch(topic, batch_dict)`` for every batch; reconnects with backoff."""

    def __init__(self, endpoint: str, on_batch: Callable[[str, dict], None], topic_filter: str = "kv@"):
        self.host, self.port = parse_endpoint(endpoint)
        if self.host == "0.0.0.0":
            self.host = "127.0.0.1"
        self.on_batch = on_batch
        self.filter = topic_filter
        self.task: Optional[asyncio.Task] = None
        self.connected = asyncio.Event()
        self.stopped = False

    def start(self):
        self.task = asyncio.get_running_loop().create_task(self._run())
        return self

    async def _run(self):
        backoff = 0.05
        while not self.stopped:
            try:
                r, w = await asyncio.open_connection(self.host, self.port)
                f = self.filter.encode()
                w.write(_frame(f))
                await w.drain()
                self.connected.set()
                backoff = 0.05
                while True:
                    n = struct.unpack("<I", await r.readexactly(4))[0]
                    topic = (await r.readexactly(n)).decode()
                    n = struct.unpack("<I", await r.readexactly(4))[0]
                    batch = msgpack.unpackb(await r.readexactly(n), raw=False, strict_map_key=False)
                    try:
                        self.on_batch(topic, batch)
                    except Exception:  # noqa: BLE001
                        log.exception("kv event handler failed")
            except (OSError, asyncio.IncompleteReadError):
                self.connected.clear()
                await asyncio.sleep(backoff)
                backoff = min(2.0, backoff * 2)
            except asyncio.CancelledError:
                return

    async def stop(self):
        self.stopped = True
        if self.task:
            self.task.cancel()
            try:
                await self.task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
