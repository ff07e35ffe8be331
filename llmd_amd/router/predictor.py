"""Latency predictor (docs/architecture/advanced/latency-predictor.md).

Two native GBDT regressors (llmd_amd._rt.GBDT): TTFT and TPOT, retrained
continuously on a sliding window of observed samples with stratified
bucketing (KV utilisation in 10 % steps x prefix-hit in 0.25 steps) so one
hot regime cannot evict the rest of the training distribution.

Features (reference order):
  TTFT: kv_cache_percentage, input_token_length, num_request_waiting,
        num_request_running, prefix_cache_score, inflight_input_tokens
  TPOT: kv_cache_percentage, input_token_length, num_request_waiting,
        num_request_running, num_tokens_generated

Deployment shapes:
  * in-process (the EPP producer owns a LatencyPredictor);
  * training server + N prediction servers sharing a model file
    (``python -m llmd_amd.router.predictor --role training|prediction``),
    HTTP API: POST /add_training_data_bulk, POST /predict, POST /predict/bulk,
    GET /model/download, GET /healthz, GET /metrics.
"""
from __future__ import annotations

import argparse
import collections
import os
import random
import threading
import time
from typing import Optional

import numpy as np

from llmd_amd import _rt_loader

TTFT_FEATS = ["kv_cache_percentage", "input_token_length", "num_request_waiting", "num_request_running",
              "prefix_cache_score", "inflight_input_tokens"]
TPOT_FEATS = ["kv_cache_percentage", "input_token_length", "num_request_waiting", "num_request_running",
              "num_tokens_generated"]


def _bucket(f: dict) -> tuple:
    return (min(9, int(float(f.get("kv_cache_percentage", 0)) * 10)),
            min(3, int(float(f.get("prefix_cache_score", 0)) * 4)))


class LatencyPredictor:
    def __init__(self, window_per_bucket: int = 2000, min_samples: int = 50, retrain_every: int = 100,
                 n_trees: int = 80, max_depth: int = 5, background: bool = False):
        self.rt = _rt_loader.rt()
        self.window = window_per_bucket
        self.min_samples = min_samples
        self.retrain_every = retrain_every
        self.n_trees, self.depth = n_trees, max_depth
        self.ttft_buckets: dict[tuple, collections.deque] = collections.defaultdict(
            lambda: collections.deque(maxlen=self.window))
        self.tpot_buckets: dict[tuple, collections.deque] = collections.defaultdict(
            lambda: collections.deque(maxlen=self.window))
        self.ttft_model = None
        self.tpot_model = None
        self.new_samples = 0
        self.lock = threading.Lock()
        self.version = 0
        self.background = background
        self._training = False

    # ------------------------------------------------------------ samples
    def add_sample(self, feats: dict, ttft_ms: Optional[float] = None, tpot_ms: Optional[float] = None):
        b = _bucket(feats)
        with self.lock:
            if ttft_ms is not None:
                self.ttft_buckets[b].append(([float(feats.get(k, 0)) for k in TTFT_FEATS], float(ttft_ms)))
            if tpot_ms is not None:
                self.tpot_buckets[b].append(([float(feats.get(k, 0)) for k in TPOT_FEATS], float(tpot_ms)))
            self.new_samples += 1
            due = self.new_samples >= self.retrain_every
        if due:
            if self.background:
                if not self._training:
                    self._training = True
                    threading.Thread(target=self._train_bg, daemon=True).start()
            else:
                self.train()

    def _train_bg(self):
        try:
            self.train()
        finally:
            self._training = False

    def num_samples(self) -> tuple[int, int]:
        return (sum(len(d) for d in self.ttft_buckets.values()), sum(len(d) for d in self.tpot_buckets.values()))

    def _fit(self, buckets):
        rows = [s for d in buckets.values() for s in d]
        if len(rows) < self.min_samples:
            return None
        X = np.asarray([r[0] for r in rows], dtype=np.float32)
        y = np.asarray([r[1] for r in rows], dtype=np.float32)
        m = self.rt.GBDT(self.n_trees, self.depth, 0.1, 5, 64, 0.0)
        m.fit(X, y)
        return m

    def train(self):
        with self.lock:
            self.new_samples = 0
            tb = {k: list(v) for k, v in self.ttft_buckets.items()}
            pb = {k: list(v) for k, v in self.tpot_buckets.items()}
        t = self._fit(tb)
        p = self._fit(pb)
        with self.lock:
            if t is not None:
                self.ttft_model = t
            if p is not None:
                self.tpot_model = p
            self.version += 1

    # ------------------------------------------------------------ predict
    @property
    def ready(self) -> bool:
        return self.ttft_model is not None and self.tpot_model is not None

    def predict(self, feats: list[dict]) -> Optional[list[dict]]:
        if not self.ready or not feats:
            return None
        Xt = np.asarray([[float(f.get(k, 0)) for k in TTFT_FEATS] for f in feats], dtype=np.float32)
        Xp = np.asarray([[float(f.get(k, 0)) for k in TPOT_FEATS] for f in feats], dtype=np.float32)
        t = self.ttft_model.predict(Xt)
        p = self.tpot_model.predict(Xp)
        return [{"ttft_ms": max(0.0, float(a)), "tpot_ms": max(0.0, float(b))} for a, b in zip(t, p)]

    # ------------------------------------------------------------ model sharing
    def save(self, path: str):
        if not self.ready:
            return
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            a, b = self.ttft_model.serialize(), self.tpot_model.serialize()
            f.write(len(a).to_bytes(8, "little") + a + b)
        os.replace(tmp, path)

    def load(self, path: str) -> bool:
        try:
            with open(path, "rb") as f:
                d = f.read()
        except OSError:
            return False
        n = int.from_bytes(d[:8], "little")
        t, p = self.rt.GBDT(), self.rt.GBDT()
        t.deserialize(d[8 : 8 + n])
        p.deserialize(d[8 + n :])
        with self.lock:
            self.ttft_model, self.tpot_model = t, p
            self.version += 1
        return True


def mape(pred: np.ndarray, y: np.ndarray) -> float:
    return float(np.mean(np.abs(pred - y) / np.maximum(np.abs(y), 1e-6)))


# ---------------------------------------------------------------- HTTP servers
def make_app(pred: LatencyPredictor, role: str, model_path: Optional[str]):
    from aiohttp import web

    async def add_bulk(req):
        body = await req.json()
        for s in body.get("entries", body.get("samples", [])):
            pred.add_sample(s, s.get("actual_ttft_ms"), s.get("actual_tpot_ms"))
        if model_path and role == "training" and pred.ready:
            pred.save(model_path)
        return web.json_response({"ok": True, "samples": pred.num_samples()})

    async def predict_one(req):
        body = await req.json()
        r = pred.predict([body])
        if r is None:
            return web.json_response({"error": "model not ready"}, status=503)
        return web.json_response(r[0])

    async def predict_bulk(req):
        body = await req.json()
        r = pred.predict(body.get("requests", []))
        if r is None:
            return web.json_response({"error": "model not ready"}, status=503)
        return web.json_response({"predictions": r})

    async def healthz(req):
        return web.json_response({"ready": pred.ready, "version": pred.version})

    async def download(req):
        if not model_path or not os.path.exists(model_path):
            return web.Response(status=404)
        return web.FileResponse(model_path)

    async def metrics(req):
        a, b = pred.num_samples()
        text = (f"latency_predictor_model_version {pred.version}\n"
                f"latency_predictor_ttft_samples {a}\nlatency_predictor_tpot_samples {b}\n")
        return web.Response(text=text)

    app = web.Application()
    app.router.add_post("/add_training_data_bulk", add_bulk)
    app.router.add_post("/predict", predict_one)
    app.router.add_post("/predict/bulk", predict_bulk)
    app.router.add_get("/healthz", healthz)
    app.router.add_get("/readyz", healthz)
    app.router.add_get("/model/download", download)
    app.router.add_get("/metrics", metrics)

    if role == "prediction" and model_path:
        async def reload_loop(app):
            async def loop():
                import asyncio
                last = 0.0
                while True:
                    try:
                        m = os.path.getmtime(model_path)
                        if m > last and pred.load(model_path):
                            last = m
                    except OSError:
                        pass
                    await asyncio.sleep(float(os.environ.get("MODEL_SYNC_INTERVAL_SEC", "10")))
            import asyncio
            app["reload"] = asyncio.get_running_loop().create_task(loop())
        app.on_startup.append(reload_loop)
    return app


def main(argv=None):
    from aiohttp import web

    p = argparse.ArgumentParser("llmd-amd latency predictor")
    p.add_argument("--role", choices=["training", "prediction", "combined"], default="combined")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--model-path", default=os.environ.get("LATENCY_MODEL_PATH"))
    p.add_argument("--min-samples", type=int, default=int(os.environ.get("LATENCY_MIN_SAMPLES", "50")))
    p.add_argument("--retrain-every", type=int, default=int(os.environ.get("LATENCY_RETRAIN_EVERY", "100")),
                   help="samples between retrains (training role)")
    a = p.parse_args(argv)
    pred = LatencyPredictor(background=True, min_samples=a.min_samples, retrain_every=a.retrain_every)
    if a.role == "prediction" and a.model_path:
        pred.load(a.model_path)
    web.run_app(make_app(pred, a.role, a.model_path), port=a.port, access_log=None)


if __name__ == "__main__":
    main()
