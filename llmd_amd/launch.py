"""Single-node launcher: the pod-group role of LeaderWorkerSet / Helm on one
8xMI355X host (reference guides/wide-ep-lws/modelserver/gpu/
vllm/base/decode.yaml:1-21,85,104-108 for the LWS env contract).

A topology YAML names the model, the router and the engine roles::

  model: llama-3-70b
  gpus: 8                      # GPUs on the host (default: all visible)
  device: cuda                 # cpu: CPU engines, no GPU assignment (the
                               # reference's docker/Dockerfile.cpu path)
  router: {port: 8000, config: <EndpointPickerConfig path or inline YAML>}
                               # mode: extproc -> the EPP as an Envoy ext_proc
                               # gRPC server on grpc_port (9002) for an external
                               # Envoy / Gateway instead of the built-in proxy
  roles:
    - name: prefill            # llm-d.ai/role label: prefill | decode | prefill-decode
      replicas: 6
      tp: 1                    # GPUs per replica (torchrun ranks for tp > 1)
      dp: 1                    # data-parallel ranks per replica (wide-EP: DP attention +
                               # --enable-expert-parallel); rank r serves port + r and
                               # is its own router endpoint (multi-port external LB)
      port: 8200               # engine port of replica 0 (+ tp x dp ... see below)
      args: ["--max-num-batched-tokens", "8192"]
      kv_transfer: true        # kvx producer/consumer by role
    - name: decode
      replicas: 2
      tp: 1
      port: 8300
      sidecar_port: 8400       # routing sidecar in front of each decode engine

  services:                    # router-side services of the well-lit paths
    - {type: predictor, port: 8100}        # latency predictor (training + prediction);
                                           # the router gets PREDICTION_SERVER_URL
    - {type: render, port: 8300}           # tokenizer / render sidecar (token-producer)
    - {type: batch-gateway, port: 8081}    # OpenAI Batch API -> router
    - {type: async-processor}              # queue-driven async dispatch -> router
    - {type: wva, port: 8080, config: {...}}   # workload variant autoscaler controller
    - {type: iro, port: 8480}              # inference resilience operator; its rank
                                           # topology map (engines, devices, DP groups,
                                           # fault-event ports) is generated from the plan
    - {type: timeslice, port: 8490}        # RL time-slicing orchestrator (llmd_amd.rl.timeslice)

Every replica gets a disjoint GPU set (``HIP_VISIBLE_DEVICES``; TP replicas
are packed onto neighbouring GPUs so TP traffic stays on direct xGMI links),
LWS-compatible env (``LWS_GROUP_SIZE`` = tp, ``LWS_LEADER_ADDRESS``,
``LWS_WORKER_INDEX``), ``POD_IP``/``POD_PORT`` (KV-event topic), and the
router gets an ``endpoints.yaml`` for file discovery with role labels.
``plan()`` is pure (testable); ``Launcher.start()/stop()`` run processes in
their own sessions and stop them by process group.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from typing import Optional

import yaml

PY = sys.executable


@dataclass
class ProcSpec:
    name: str
    cmd: list[str]
    env: dict[str, str] = field(default_factory=dict)
    gpus: list[int] = field(default_factory=list)
    port: Optional[int] = None
    role: str = ""
    health: str = "/health"  # readiness path polled by wait_ready


def _kv_transfer(role: str) -> str:
    r = {"prefill": "kv_producer", "decode": "kv_consumer"}.get(role, "kv_both")
    return json.dumps({"kv_connector": "KvxConnector", "kv_role": r})


def plan(topo: dict, workdir: str) -> tuple[list[ProcSpec], dict]:
    """Returns (process specs, router endpoints doc)."""
    cpu = topo.get("device", "cuda") == "cpu"
    n_gpus = 0 if cpu else int(topo.get("gpus", 8))
    model = topo["model"]
    free = list(range(n_gpus))
    procs: list[ProcSpec] = []
    endpoints = []
    master_port = int(topo.get("master_port_base", 29600))
    ev_next = 0  # KV-event ports handed out so far (one per engine process / DP rank)
    node = str(topo.get("node_name", "localhost"))
    iro_engines = []  # rank topology map for the resilience operator (nodeName + devices -> engine)
    for role in topo.get("roles", []):
        name, tp, dp = role["name"], int(role.get("tp", 1)), int(role.get("dp", 1))
        ranks = tp * dp
        for i in range(int(role.get("replicas", 1))):
            if cpu:
                gpus = []
            elif len(free) < ranks:
                raise ValueError(f"not enough GPUs for {name} replica {i} (tp={tp}, dp={dp}, free={free})")
            else:
                gpus, free = free[:ranks], free[ranks:]
            port = int(role.get("port", 8200)) + i * dp  # DP rank r of the replica serves port + r
            args = ["--model", model, "--port", str(port), "--tensor-parallel-size", str(tp)] + \
                (["--data-parallel-size", str(dp)] if dp > 1 else []) + \
                (["--device", "cpu"] if cpu else []) + [str(x) for x in role.get("args", [])]
            if role.get("kv_transfer", name in ("prefill", "decode")):
                args += ["--kv-transfer-config", _kv_transfer(name)]
            ev_port = int(role.get("kv_events_port", 5556)) + ev_next  # DP rank r publishes on ev_port + r
            if role.get("kv_events", False):
                args += ["--kv-events-config", json.dumps(
                    {"enable_kv_cache_events": True, "publisher": "zmq", "endpoint": f"tcp://*:{ev_port}"})]
                ev_next += dp
            server = ["-m", "llmd_amd.serving.api_server"] + args
            if ranks > 1:
                cmd = [PY, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                       "--master-addr=127.0.0.1", f"--master-port={master_port}"] + server
                master_port += 1
            else:
                cmd = [PY] + server
            env = {"HIP_VISIBLE_DEVICES": ",".join(map(str, gpus)) if not cpu else "", "LWS_GROUP_SIZE": str(tp),
                   "LWS_LEADER_ADDRESS": "127.0.0.1", "LWS_WORKER_INDEX": "0", "POD_IP": "127.0.0.1",
                   "POD_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
            rid = f"{name}-{i}"
            procs.append(ProcSpec(rid, cmd, env, gpus, port, name))
            front = port
            if name == "decode" and role.get("sidecar_port"):
                front = int(role["sidecar_port"]) + i
                procs.append(ProcSpec(rid + "-sidecar",
                                      [PY, "-m", "llmd_amd.sidecar.routing_sidecar", "--port", str(front),
                                       "--vllm-port", str(port), "--connector", role.get("connector", "nixlv2")],
                                      {}, [], front, "sidecar"))
            labels = {"llm-d.ai/role": name if name in ("prefill", "decode", "encode") else "prefill-decode",
                      "llm-d.ai/model": model}
            for r in range(dp):  # one router endpoint per DP rank
                lab = dict(labels)
                if role.get("kv_events", False):
                    lab["llm-d.ai/kv-events-port"] = str(ev_port + r)
                ep_name = rid if dp == 1 else f"{rid}-dp{r}"
                endpoints.append({"name": ep_name, "address": "127.0.0.1", "port": front + r, "labels": lab,
                                  "metricsPort": port + r})
                iro = {"name": ep_name, "url": f"http://127.0.0.1:{port + r}", "nodeName": node,
                       "devices": gpus[r * tp:(r + 1) * tp],
                       "endpoints": [{"address": "127.0.0.1", "port": front + r}]}
                if dp > 1:  # wide-EP DP ranks step in lockstep: one recovery group
                    iro["group"] = rid
                if role.get("kv_events", False):
                    iro["faultEvents"] = f"tcp://127.0.0.1:{ev_port + r}"
                iro_engines.append(iro)
                if r:
                    procs.append(ProcSpec(ep_name, [], {}, [], port + r, name + "-dp-rank"))
    doc = {"endpoints": endpoints}
    r = topo.get("router")
    router_env: dict[str, str] = {}
    rport_http = int((r or {}).get("port", 8000))
    for svc in topo.get("services", []) or []:
        spec = _service(svc, model, workdir, rport_http, iro_engines)
        procs.append(spec)
        if svc["type"] == "predictor":
            router_env["PREDICTION_SERVER_URL"] = f"http://127.0.0.1:{spec.port}"
            router_env["TRAINING_SERVER_URL"] = f"http://127.0.0.1:{spec.port}"
    if r:
        ep_file = os.path.join(workdir, "endpoints.yaml")
        if r.get("mode", "proxy") == "extproc":
            cmd = [PY, "-m", "llmd_amd.router.extproc", "--grpc-port", str(r.get("grpc_port", 9002)),
                   "--grpc-health-port", str(r.get("grpc_health_port", 9003)),
                   "--metrics-port", str(r.get("metrics_port", 9090)), "--endpoints-file", ep_file]
        else:
            cmd = [PY, "-m", "llmd_amd.router.proxy", "--port", str(r.get("port", 8000)),
                   "--endpoints-file", ep_file]
            if int(r.get("workers", 1)) > 1:  # native relay threads in front of one EPP process
                cmd += ["--workers", str(int(r["workers"])), "--metrics-port", str(r.get("metrics_port", 9090))]
        conf = r.get("config")
        if conf:
            if os.path.exists(str(conf)):
                cmd += ["--config-file", str(conf)]
            else:
                cmd += ["--config-text", conf if isinstance(conf, str) else yaml.safe_dump(conf)]
        rport = int(r.get("grpc_port", 9002)) if r.get("mode") == "extproc" else int(r.get("port", 8000))
        procs.append(ProcSpec("router", cmd, router_env, [], rport, "router"))
    return procs, doc


SERVICES = {"predictor": "llmd_amd.router.predictor", "render": "llmd_amd.serving.render_server",
            "batch-gateway": "llmd_amd.batch.gateway", "async-processor": "llmd_amd.batch.async_processor",
            "wva": "llmd_amd.autoscale.controller", "iro": "llmd_amd.resilience.operator",
            "timeslice": "llmd_amd.rl.timeslice"}


def _service(svc: dict, model: str, workdir: str, router_port: int, engines: Optional[list] = None) -> ProcSpec:
    """Router-side service of a well-lit path as a process spec."""
    t = svc["type"]
    if t not in SERVICES:
        raise ValueError(f"unknown service type {t!r}; known: {sorted(SERVICES)}")
    port = svc.get("port")
    cmd = [PY, "-m", SERVICES[t]]
    gw = f"http://127.0.0.1:{router_port}"
    if t == "predictor":
        port = int(port or 8100)
        cmd += ["--port", str(port), "--role", svc.get("role", "combined")]
        if svc.get("model_path"):
            cmd += ["--model-path", str(svc["model_path"])]
    elif t == "render":
        port = int(port or 8300)
        cmd += ["--port", str(port), "--model", model]
    elif t == "batch-gateway":
        port = int(port or 8081)
        cmd += ["--port", str(port), "--gateway-url", gw, "--root", svc.get("root", os.path.join(workdir, "batch"))]
    elif t == "async-processor":
        port = None
        cmd += ["--igw-base-url", gw, "--db", svc.get("db", os.path.join(workdir, "async-mq.db"))]
    elif t == "wva":
        port = int(port or 8080)
        conf = dict(svc.get("config") or {})
        conf.setdefault("endpointsFile", os.path.join(workdir, "endpoints.yaml"))
        conf.setdefault("eppMetricsUrl", f"{gw}/metrics")
        path = os.path.join(workdir, "wva-config.yaml")
        if workdir and not workdir.startswith("<") and os.path.isdir(workdir):
            with open(path, "w") as f:
                yaml.safe_dump(conf, f)
        cmd += ["--config", path, "--metrics-bind-address", f":{port}"]
    elif t == "iro":
        port = int(port or 8480)
        conf = dict(svc.get("config") or {})
        conf.setdefault("recoveryRequestsDir", os.path.join(workdir, "recoveryrequests"))
        conf.setdefault("endpointsFile", os.path.join(workdir, "endpoints.yaml"))
        conf.setdefault("engines", list(engines or []))
        path = os.path.join(workdir, "iro-config.yaml")
        if workdir and not workdir.startswith("<") and os.path.isdir(workdir):
            with open(path, "w") as f:
                yaml.safe_dump(conf, f)
        cmd += ["--config", path, "--port", str(port)]
    elif t == "timeslice":
        port = int(port or 8490)
        cmd += ["--port", str(port)]
    cmd += [str(a) for a in svc.get("args", [])]
    health = {"predictor": "/healthz", "batch-gateway": "/v1/batches", "wva": "/metrics",
              "iro": "/healthz", "timeslice": "/healthz"}.get(t, "/health")
    return ProcSpec(svc.get("name", t), cmd, dict(svc.get("env") or {}), [], port, "service", health)


class Launcher:
    def __init__(self, topo: dict, workdir: Optional[str] = None, log_dir: Optional[str] = None):
        self.topo = topo
        self.workdir = workdir or tempfile.mkdtemp(prefix="llmd-launch-")
        self.log_dir = log_dir or self.workdir
        self.specs, self.endpoints = plan(topo, self.workdir)
        self.procs: list[tuple[ProcSpec, subprocess.Popen]] = []

    def start(self):
        with open(os.path.join(self.workdir, "endpoints.yaml"), "w") as f:
            yaml.safe_dump(self.endpoints, f)
        for s in self.specs:
            if not s.cmd:  # a DP rank > 0: served by its replica's torchrun group (started above)
                continue
            env = dict(os.environ, **s.env)
            log = open(os.path.join(self.log_dir, f"{s.name}.log"), "w")
            p = subprocess.Popen(s.cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
            self.procs.append((s, p))
        return self

    def wait_ready(self, timeout: float = 1800.0) -> bool:
        import urllib.request

        t0 = time.time()
        pending = [s for s in self.specs if s.port and s.role != "router"]
        while pending and time.time() - t0 < timeout:
            for s in list(pending):
                try:
                    with urllib.request.urlopen(f"http://127.0.0.1:{s.port}{s.health}", timeout=2) as r:
                        if r.status == 200:
                            pending.remove(s)
                except OSError:
                    pass
            if any(p.poll() is not None for _, p in self.procs):
                return False
            time.sleep(1.0)
        return not pending

    def stop(self, grace: float = 30.0):
        for s, p in reversed(self.procs):
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t0 = time.time()
        for s, p in self.procs:
            while p.poll() is None and time.time() - t0 < grace:
                time.sleep(0.1)
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        self.procs.clear()


def main(argv=None):
    ap = argparse.ArgumentParser("llmd-launch")
    ap.add_argument("topology", help="topology YAML")
    ap.add_argument("--dry-run", action="store_true", help="print the process plan and exit")
    ap.add_argument("--log-dir", default=None)
    a = ap.parse_args(argv)
    with open(a.topology) as f:
        topo = yaml.safe_load(f)
    if a.dry_run:
        specs, doc = plan(topo, "<workdir>")
        for s in specs:
            print(f"{s.name:18} gpus={s.gpus} port={s.port} env={s.env.get('HIP_VISIBLE_DEVICES', '')}\n"
                  f"    {' '.join(s.cmd) or '(DP rank of the replica above)'}")
        print(yaml.safe_dump(doc))
        return
    la = Launcher(topo, log_dir=a.log_dir).start()
    try:
        ok = la.wait_ready()
        print("all engines ready" if ok else "an engine exited during start-up; see logs in " + la.log_dir,
              flush=True)
        while ok and all(p.poll() is None for _, p in la.procs):
            time.sleep(1.0)
    except KeyboardInterrupt:
        pass
    finally:
        la.stop()


if __name__ == "__main__":
    main()
