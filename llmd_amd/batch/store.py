"""Batch Gateway storage layer (reference
docs/architecture/advanced/batch/batch-gateway.md "Storage Layer").

Single-node deployment: one SQLite database holds job/file metadata, the
priority queue (ordered by SLO deadline, i.e. ``created_at + completion
window``) and the event channel (cancel requests); file contents live on a
filesystem under ``<root>/<sha256(tenant)[:16]>/<file_id>`` so paths cannot be
enumerated across tenants. All queries are filtered by tenant id.
"""
from __future__ import annotations

import hashlib
import json
import os
import sqlite3
import threading
import time
import uuid
from typing import Optional

_SCHEMA = """
CREATE TABLE IF NOT EXISTS files (
  id TEXT PRIMARY KEY, tenant TEXT NOT NULL, filename TEXT, purpose TEXT,
  bytes INTEGER, created_at INTEGER, expires_at INTEGER, path TEXT);
CREATE TABLE IF NOT EXISTS batches (
  id TEXT PRIMARY KEY, tenant TEXT NOT NULL, body TEXT NOT NULL);
CREATE TABLE IF NOT EXISTS queue (
  batch_id TEXT PRIMARY KEY, priority REAL NOT NULL, enqueued_at REAL NOT NULL);
CREATE TABLE IF NOT EXISTS events (
  batch_id TEXT NOT NULL, kind TEXT NOT NULL, at REAL NOT NULL);
CREATE INDEX IF NOT EXISTS files_tenant ON files(tenant);
CREATE INDEX IF NOT EXISTS batches_tenant ON batches(tenant);
"""

WINDOWS = {"s": 1, "m": 60, "h": 3600, "d": 86400}


def parse_window(w: str) -> int:
    w = str(w).strip()
    if w and w[-1] in WINDOWS and w[:-1].isdigit():
        return int(w[:-1]) * WINDOWS[w[-1]]
    raise ValueError(f"invalid completion_window {w!r}")


class Store:
    """Thread-safe metadata + queue + file store."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(os.path.join(root, "files"), exist_ok=True)
        self.db = sqlite3.connect(os.path.join(root, "batch.db"), check_same_thread=False,
                                  isolation_level=None)
        self.db.execute("PRAGMA journal_mode=WAL")
        self.db.executescript(_SCHEMA)
        self.lock = threading.RLock()

    # ----------------------------------------------------------------- files
    def _file_path(self, tenant: str, fid: str) -> str:
        d = os.path.join(self.root, "files", hashlib.sha256(tenant.encode()).hexdigest()[:16])
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, fid)

    def put_file(self, tenant: str, filename: str, purpose: str, data: bytes,
                 expires_after: Optional[int] = None) -> dict:
        fid = "file-" + uuid.uuid4().hex
        path = self._file_path(tenant, fid)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
        now = int(time.time())
        exp = now + expires_after if expires_after else None
        with self.lock:
            self.db.execute("INSERT INTO files VALUES (?,?,?,?,?,?,?,?)",
                            (fid, tenant, filename, purpose, len(data), now, exp, path))
        return self.file_obj(tenant, fid)

    def file_obj(self, tenant: str, fid: str) -> Optional[dict]:
        with self.lock:
            r = self.db.execute("SELECT id, filename, purpose, bytes, created_at, expires_at FROM files "
                                "WHERE id=? AND tenant=?", (fid, tenant)).fetchone()
        if r is None:
            return None
        return {"id": r[0], "object": "file", "bytes": r[3], "created_at": r[4], "expires_at": r[5],
                "filename": r[1], "purpose": r[2], "status": "processed"}

    def list_files(self, tenant: str, purpose: Optional[str] = None, limit: int = 10000) -> list[dict]:
        q = "SELECT id FROM files WHERE tenant=?" + (" AND purpose=?" if purpose else "") + \
            " ORDER BY created_at DESC, rowid DESC LIMIT ?"
        args = (tenant, purpose, limit) if purpose else (tenant, limit)
        with self.lock:
            ids = [r[0] for r in self.db.execute(q, args).fetchall()]
        return [self.file_obj(tenant, i) for i in ids]

    def file_content(self, tenant: str, fid: str) -> Optional[bytes]:
        with self.lock:
            r = self.db.execute("SELECT path FROM files WHERE id=? AND tenant=?", (fid, tenant)).fetchone()
        if r is None or not os.path.exists(r[0]):
            return None
        with open(r[0], "rb") as f:
            return f.read()

    def delete_file(self, tenant: str, fid: str) -> bool:
        with self.lock:
            r = self.db.execute("SELECT path FROM files WHERE id=? AND tenant=?", (fid, tenant)).fetchone()
            if r is None:
                return False
            self.db.execute("DELETE FROM files WHERE id=?", (fid,))
        try:
            os.remove(r[0])
        except OSError:
            pass
        return True

    def open_output(self, tenant: str, fid: str) -> str:
        """Path for a processor-written output file (registered on finalize)."""
        return self._file_path(tenant, fid)

    def register_file(self, tenant: str, fid: str, filename: str, purpose: str, path: str) -> dict:
        n = os.path.getsize(path)
        with self.lock:
            self.db.execute("INSERT OR REPLACE INTO files VALUES (?,?,?,?,?,?,?,?)",
                            (fid, tenant, filename, purpose, n, int(time.time()), None, path))
        return self.file_obj(tenant, fid)

    # --------------------------------------------------------------- batches
    def put_batch(self, tenant: str, b: dict):
        with self.lock:
            self.db.execute("INSERT OR REPLACE INTO batches VALUES (?,?,?)", (b["id"], tenant, json.dumps(b)))

    def get_batch(self, tenant: Optional[str], bid: str) -> Optional[dict]:
        with self.lock:
            if tenant is None:
                r = self.db.execute("SELECT body, tenant FROM batches WHERE id=?", (bid,)).fetchone()
            else:
                r = self.db.execute("SELECT body, tenant FROM batches WHERE id=? AND tenant=?",
                                    (bid, tenant)).fetchone()
        if r is None:
            return None
        b = json.loads(r[0])
        b["_tenant"] = r[1]
        return b

    def update_batch(self, bid: str, **fields) -> Optional[dict]:
        with self.lock:
            r = self.db.execute("SELECT body FROM batches WHERE id=?", (bid,)).fetchone()
            if r is None:
                return None
            b = json.loads(r[0])
            for k, v in fields.items():
                if k == "request_counts":
                    b.setdefault("request_counts", {}).update(v)
                else:
                    b[k] = v
            self.db.execute("UPDATE batches SET body=? WHERE id=?", (json.dumps(b), bid))
        return b

    def list_batches(self, tenant: str, after: Optional[str] = None, limit: int = 20) -> list[dict]:
        with self.lock:
            rows = self.db.execute("SELECT body FROM batches WHERE tenant=? ORDER BY rowid DESC",
                                   (tenant,)).fetchall()
        out = [json.loads(r[0]) for r in rows]
        if after:
            ids = [b["id"] for b in out]
            if after in ids:
                out = out[ids.index(after) + 1:]
        return out[:limit]

    def batches_in_status(self, *statuses) -> list[dict]:
        with self.lock:
            rows = self.db.execute("SELECT body, tenant FROM batches").fetchall()
        res = []
        for body, tenant in rows:
            b = json.loads(body)
            if b.get("status") in statuses:
                b["_tenant"] = tenant
                res.append(b)
        return res

    def delete_batch(self, bid: str):
        with self.lock:
            self.db.execute("DELETE FROM batches WHERE id=?", (bid,))
            self.db.execute("DELETE FROM queue WHERE batch_id=?", (bid,))
            self.db.execute("DELETE FROM events WHERE batch_id=?", (bid,))

    # ---------------------------------------------------------------- queue
    def enqueue(self, bid: str, priority: float):
        with self.lock:
            self.db.execute("INSERT OR REPLACE INTO queue VALUES (?,?,?)", (bid, priority, time.time()))

    def dequeue(self) -> Optional[tuple[str, float]]:
        """Pop the job with the earliest deadline (lowest score)."""
        with self.lock:
            r = self.db.execute("SELECT batch_id, enqueued_at FROM queue ORDER BY priority, enqueued_at "
                                "LIMIT 1").fetchone()
            if r is None:
                return None
            self.db.execute("DELETE FROM queue WHERE batch_id=?", (r[0],))
        return r[0], r[1]

    def queue_len(self) -> int:
        with self.lock:
            return self.db.execute("SELECT COUNT(*) FROM queue").fetchone()[0]

    # --------------------------------------------------------------- events
    def post_event(self, bid: str, kind: str):
        with self.lock:
            self.db.execute("INSERT INTO events VALUES (?,?,?)", (bid, kind, time.time()))

    def has_event(self, bid: str, kind: str) -> bool:
        with self.lock:
            return self.db.execute("SELECT 1 FROM events WHERE batch_id=? AND kind=? LIMIT 1",
                                   (bid, kind)).fetchone() is not None

    # ------------------------------------------------------------------- gc
    def expired_files(self, now: float) -> list[tuple[str, str]]:
        with self.lock:
            return self.db.execute("SELECT tenant, id FROM files WHERE expires_at IS NOT NULL AND expires_at < ?",
                                   (now,)).fetchall()

    def close(self):
        with self.lock:
            self.db.close()
