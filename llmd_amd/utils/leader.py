"""Lease-based leader election for active-passive HA (the EPP's
``--ha-enable-leader-election`` when replicas > 1,
docs/architecture/core/router/epp/configuration.md:455-459; WVA
``--leader-elect --leader-election-lease-duration 60s
--leader-election-renew-deadline 50s``,
docs/architecture/advanced/autoscaling/wva.md:397-400).

The Kubernetes Lease object becomes a small JSON record in a file every
replica can reach (one node, or a shared volume):
``{"holder", "acquire_time", "renew_time", "lease_duration_s", "transitions"}``.
Every read-modify-write of the record happens under an exclusive ``flock`` on
a side lock file, so two candidates never both see an expired lease and both
take it. A candidate

* acquires the lease when it is free, expired (``renew_time +
  lease_duration`` in the past) or already its own;
* renews it every ``retry_period`` while leading;
* steps down (``on_stopped_leading``) when it could not renew for
  ``renew_deadline`` (a stalled leader must stop acting before a standby may
  take over: ``renew_deadline < lease_duration``);
* releases it on a clean ``stop()`` so a standby takes over at once instead of
  after a full lease duration.

A leader that dies without releasing is replaced after ``lease_duration``.
Time is wall-clock (``time.time``): candidates in different processes compare
``renew_time`` against their own clocks, as client-go does.
"""
from __future__ import annotations

import fcntl
import json
import logging
import os
import socket
import threading
import time
import uuid
from typing import Callable, Optional

log = logging.getLogger("llmd.leader")


class LeaseElector:
    def __init__(self, lease_file: str, identity: Optional[str] = None, lease_duration: float = 15.0,
                 renew_deadline: float = 10.0, retry_period: float = 2.0,
                 on_started_leading: Optional[Callable[[], None]] = None,
                 on_stopped_leading: Optional[Callable[[], None]] = None):
        if not 0 < retry_period < renew_deadline < lease_duration:
            raise ValueError("leader election needs 0 < retry_period < renew_deadline < lease_duration")
        self.path = lease_file
        self.lock_path = lease_file + ".lock"
        self.identity = identity or f"{socket.gethostname()}-{os.getpid()}-{uuid.uuid4().hex[:6]}"
        self.lease_duration, self.renew_deadline, self.retry_period = lease_duration, renew_deadline, retry_period
        self.on_started, self.on_stopped = on_started_leading, on_stopped_leading
        self._leader = False
        self._last_renew = 0.0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        d = os.path.dirname(os.path.abspath(lease_file))
        os.makedirs(d, exist_ok=True)

    # ------------------------------------------------------------ record I/O
    def _read(self) -> dict:
        try:
            with open(self.path) as f:
                return json.load(f)
        except (FileNotFoundError, json.JSONDecodeError):
            return {}

    def _write(self, rec: dict):
        tmp = f"{self.path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, self.path)  # atomic for readers that skip the lock

    def _locked(self, fn):
        with open(self.lock_path, "a+") as lf:
            fcntl.flock(lf, fcntl.LOCK_EX)
            try:
                return fn()
            finally:
                fcntl.flock(lf, fcntl.LOCK_UN)

    # ------------------------------------------------------------ protocol
    def try_acquire_or_renew(self) -> bool:
        """One election round; True if this candidate holds the lease after it."""
        def rnd():
            now = time.time()
            rec = self._read()
            holder = rec.get("holder")
            expired = now > float(rec.get("renew_time", 0)) + float(rec.get("lease_duration_s", 0))
            if holder and holder != self.identity and not expired:
                return False
            if holder != self.identity:
                rec = {"holder": self.identity, "acquire_time": now,
                       "transitions": int(rec.get("transitions", 0)) + (1 if holder else 0)}
            rec["renew_time"] = now
            rec["lease_duration_s"] = self.lease_duration
            self._write(rec)
            return True
        try:
            return self._locked(rnd)
        except OSError as e:  # unreachable lease store: cannot renew
            log.warning("lease %s unavailable: %s", self.path, e)
            return False

    def release(self):
        def rel():
            rec = self._read()
            if rec.get("holder") == self.identity:
                rec["holder"] = ""
                rec["renew_time"] = 0
                self._write(rec)
        try:
            self._locked(rel)
        except OSError:
            pass

    def holder(self) -> Optional[str]:
        rec = self._read()
        if not rec.get("holder") or time.time() > float(rec.get("renew_time", 0)) + float(
                rec.get("lease_duration_s", 0)):
            return None
        return rec["holder"]

    @property
    def is_leader(self) -> bool:
        return self._leader

    def tick(self):
        """One retry period's worth of work (the background loop calls this)."""
        now = time.time()
        ok = self.try_acquire_or_renew()
        if ok:
            self._last_renew = now
            if not self._leader:
                self._leader = True
                log.info("%s became leader of %s", self.identity, self.path)
                if self.on_started:
                    self.on_started()
        elif self._leader and now - self._last_renew > self.renew_deadline:
            self._step_down("renew deadline exceeded")
        elif self._leader and not ok:
            # someone else holds a valid lease (e.g. ours expired while stalled)
            rec = self._read()
            if rec.get("holder") and rec.get("holder") != self.identity:
                self._step_down(f"lease taken by {rec.get('holder')}")

    def _step_down(self, why: str):
        self._leader = False
        log.warning("%s stopped leading %s: %s", self.identity, self.path, why)
        if self.on_stopped:
            self.on_stopped()

    def _loop(self):
        while not self._stop.is_set():
            self.tick()
            self._stop.wait(self.retry_period)

    def start(self) -> "LeaseElector":
        self._thread = threading.Thread(target=self._loop, daemon=True, name="leader-election")
        self._thread.start()
        return self

    def stop(self, release: bool = True):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        if self._leader:
            self._leader = False
            if self.on_stopped:
                self.on_stopped()
        if release:
            self.release()
