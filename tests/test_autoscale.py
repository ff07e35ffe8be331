"""WVA autoscaler (C33) + HPA signal math (C32): analyzers, optimizers,
enforcer, scale-from-zero, Kalman tuner, M/M/1/K capacity, process actuator."""
import sys

from llmd_amd.autoscale.wva import (CostAwareOptimizer, GreedyByScoreOptimizer, KalmanTuner,
                                    PercentageSaturationAnalyzer, ProcessActuator, ReplicaMetrics, SLOAnalyzer,
                                    ScalingRequest, TokenSaturationAnalyzer, Variant, WVAEngine,
                                    hpa_desired_replicas, mm1k_latency)


def _v(name, cost, cur, kv, q, mn=1, mx=4, **kw):
    v = Variant(name, "m", mn, mx, cost, current=cur, desired=cur)
    v.replicas = [ReplicaMetrics(f"{name}-{i}", kv_usage=kv, queue_len=q, num_gpu_blocks=1000, block_size=16, **kw)
                  for i in range(cur)]
    return v


def test_percentage_analyzer_up_down_blocked():
    a = PercentageSaturationAnalyzer()
    assert a.analyze("m", [_v("a", 5, 2, 0.75, 0)]).required == 1  # spare kv 0.05 < 0.10
    assert a.analyze("m", [_v("a", 5, 2, 0.1, 4)]).required == 1   # spare queue 1 < 3
    r = a.analyze("m", [_v("a", 5, 3, 0.2, 0)])
    assert r.required == 0 and r.spare == 1                        # 3->2 keeps headroom
    assert a.analyze("m", [_v("a", 5, 2, 0.6, 0)]).spare == 0      # 0.6*2=1.2 would saturate
    busy = _v("a", 5, 2, 0.75, 0)
    busy.desired = 3                                                # transitioning blocks scaling
    r = a.analyze("m", [busy])
    assert r.required == 0 and r.spare == 0


def test_cost_aware_optimizer():
    cheap, dear = _v("cheap", 5, 1, 0.9, 0, mx=2), _v("dear", 15, 1, 0.9, 0, mn=0, mx=5)
    opt = CostAwareOptimizer()
    assert opt.optimize(ScalingRequest("m", required=1), [cheap, dear]) == {"cheap": 2, "dear": 1}
    assert opt.optimize(ScalingRequest("m", required=3), [cheap, dear]) == {"cheap": 2, "dear": 3}
    assert opt.optimize(ScalingRequest("m", spare=1), [cheap, dear]) == {"cheap": 1, "dear": 0}


def test_token_analyzer_k1_k2_chain():
    a = TokenSaturationAnalyzer()
    v = _v("a", 5, 2, 0.5, 0, avg_input_tokens=1000, avg_output_tokens=200, max_num_batched_tokens=2048,
           max_num_seqs=256)
    r0 = v.replicas[0]
    k1 = r0.kv_tokens * 0.8
    n = min(256, 2048 * 200 / 1200)
    assert abs(a.k2(v, r0) - n * 1100) < 1e-6          # derived from deployment args
    assert a.capacity(v, r0) == min(k1, n * 1100)
    sat = ReplicaMetrics("x", kv_usage=0.4, queue_len=9, num_gpu_blocks=1000, block_size=16,
                         avg_input_tokens=1000, avg_output_tokens=200)
    assert a.k2(v, sat) == sat.tokens_in_use            # observed (queue saturated)
    assert a.k2(v, r0) == sat.tokens_in_use             # historical now wins over derived
    req = a.analyze("m", [v], epp_queue=10)
    assert req.unit == "tokens" and req.required > 0    # EPP queue demand pushes scale-up


def test_kalman_tuner_learns_parameters():
    true = KalmanTuner(theta0=(0.008, 2e-4, 3e-9))
    t = KalmanTuner()
    for i in range(300):
        n, isl, osl = 1 + (i * 7) % 60, 200 + (i * 131) % 3000, 50 + (i * 17) % 400
        t.update(n, isl, osl, true.prefill_time(isl), true.iter_time(n, isl + osl / 2))
    for n, ctx in ((1, 500), (32, 2000), (64, 3000)):
        assert abs(t.iter_time(n, ctx) - true.iter_time(n, ctx)) / true.iter_time(n, ctx) < 0.05
    assert abs(t.prefill_time(1000) - true.prefill_time(1000)) / true.prefill_time(1000) < 0.05


def test_mm1k_and_slo_analyzer():
    an = SLOAnalyzer(targetTTFT=500, targetITL=50, max_batch=64)
    an.tuner = KalmanTuner(theta0=(0.01, 1e-4, 2e-9))
    t_lo = mm1k_latency(0.1, an.tuner, 1000, 100, 64)
    t_hi = mm1k_latency(5.0, an.tuner, 1000, 100, 64)
    assert t_hi[0] > t_lo[0] and t_hi[1] >= t_lo[1]   # latency grows with load
    mr = an.max_rate(1000, 100)
    ttft, itl, loss = mm1k_latency(mr, an.tuner, 1000, 100, 64)
    assert ttft <= 0.5 + 1e-6 and itl <= 0.05 + 1e-6 and mr > 0
    v = _v("a", 5, 2, 0.3, 0, arrival_rate=mr * 1.6, avg_input_tokens=1000, avg_output_tokens=100)
    an.tuning = False
    assert an.analyze("m", [v]).desired_replicas == 4  # 2 replicas x 1.6 x rate -> ceil(3.2)


def test_enforcer_and_scale_from_zero():
    eng = WVAEngine({"enable_scale_to_zero": True, "retention_period": "10m"})
    a = _v("a", 5, 1, 0.1, 0, mn=0)
    d = eng.step({"m": [a]}, requests_in_retention={"m": 0})
    assert d["m"] == {"a": 0}
    a.current, a.replicas = 0, []
    eng.fast_step({"m": [a]}, {"m": 3})
    assert a.desired == 1
    eng2 = WVAEngine({})
    b = _v("b", 5, 0, 0, 0, mn=0)
    assert eng2.step({"m": [b]})["m"] == {"b": 1}   # min one replica when scale-to-zero is off


def test_greedy_by_score_budget():
    p1 = [_v("a", 5, 1, 0.9, 0, mx=8)]
    p2 = [_v("b", 5, 1, 0.9, 0, mx=8)]
    opt = GreedyByScoreOptimizer(gpu_budget=5)
    r1, r2 = ScalingRequest("m1", required=4, priority=2.0), ScalingRequest("m2", required=4, priority=1.0)
    alloc = opt.optimize_all({"m1": (r1, p1), "m2": (r2, p2)})
    total = alloc["m1"]["a"] + alloc["m2"]["b"]
    assert total == 5 and alloc["m1"]["a"] > alloc["m2"]["b"]


def test_hpa_math():
    assert hpa_desired_replicas(2, 20, 5, "Value") == 8
    assert hpa_desired_replicas(4, 40, 10, "AverageValue") == 4        # within tolerance
    assert hpa_desired_replicas(4, 80, 10, "AverageValue") == 8
    assert hpa_desired_replicas(0, 3, 5, "Value") == 1                 # scale from zero


def test_process_actuator(tmp_path):
    act = ProcessActuator(3, lambda v, gpus, i: [sys.executable, "-c", "import time; time.sleep(60)"])
    v = Variant("a", "m", 0, 3, 5.0, gpus_per_replica=1)
    act.scale(v, 2)
    assert v.current == 2 and act.free == [2]
    act.scale(v, 5)
    assert v.current == 3 and act.free == []
    act.scale(v, 1)
    assert v.current == 1 and act.free == [1, 2]
    act.shutdown()


def test_wva_controller_scales_sim_replicas(tmp_path):
    """The single-node WVA controller (autoscale/controller.py) closes the loop
    the reference leaves to HPA: VariantAutoscaling objects + launch recipes ->
    scrape replica /metrics -> saturation analyzer -> cost-aware optimizer ->
    process actuation -> router endpoints file; here with simulator replicas
    (llmd_amd/sim) as the engines: a queue builds on one replica -> scale to 2
    (both in endpoints.yaml, wva_desired_replicas = 2); the load ends -> back
    to minReplicas."""
    import json
    import socket
    import sys
    import threading
    import time
    import urllib.request

    import yaml

    from llmd_amd.autoscale.controller import WVAController

    def free_port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]

    base = free_port()
    while True:  # two consecutive free ports
        try:
            with socket.socket() as s:
                s.bind(("127.0.0.1", base + 1))
            break
        except OSError:
            base = free_port()
    ep_file = str(tmp_path / "endpoints.yaml")
    cfg = {"interval": "0.5s", "gpus": 8, "endpointsFile": ep_file,
           "scalingConfig": {"kvCacheThreshold": 0.8, "queueLengthThreshold": 5, "kvSpareTrigger": 0.1,
                             "queueSpareTrigger": 3},
           "variantAutoscalings": [{
               "apiVersion": "llmd.ai/v1alpha1", "kind": "VariantAutoscaling", "metadata": {"name": "sim-tp1"},
               "spec": {"modelID": "sim-model", "minReplicas": 1, "maxReplicas": 2, "variantCost": "5.0",
                        "scaleTargetRef": {"kind": "EngineGroup", "name": "sim-tp1"}},
               "launch": {"cpu": True, "portBase": base}}]}

    def sim_cmd(v, ln, port):
        return [sys.executable, "-m", "llmd_amd.sim.server", "--port", str(port), "--max-num-seqs", "2",
                "--decode-step-ms", "40", "--model", "sim-model"]

    ctl = WVAController(cfg, launch_cmd=sim_cmd)

    def wait_for(pred, t=60):
        t0 = time.time()
        while time.time() - t0 < t:
            if pred():
                return True
            time.sleep(0.2)
        return False

    def n_endpoints():
        try:
            return len(yaml.safe_load(open(ep_file))["endpoints"])
        except (OSError, TypeError, KeyError):
            return -1

    ctl.start()
    try:
        v = ctl.variants["sim-tp1"]
        assert v.current == 1
        assert wait_for(lambda: n_endpoints() == 1), "replica 0 never became ready"

        def req():
            body = json.dumps({"model": "sim-model", "prompt": "hello " * 30, "max_tokens": 120}).encode()
            r = urllib.request.Request(f"http://127.0.0.1:{base}/v1/completions", data=body,
                                       headers={"content-type": "application/json"})
            urllib.request.urlopen(r, timeout=120).read()

        load = [threading.Thread(target=req, daemon=True) for _ in range(10)]
        for t in load:
            t.start()
        assert wait_for(lambda: v.current == 2, 30), ctl.render_metrics()
        assert wait_for(lambda: n_endpoints() == 2, 30)
        assert 'wva_desired_replicas{variant_name="sim-tp1",exported_namespace="default",model_id="sim-model"} 2' \
            in ctl.render_metrics()
        for t in load:
            t.join(timeout=120)
        assert wait_for(lambda: v.current == 1, 60), ctl.render_metrics()
        assert wait_for(lambda: n_endpoints() == 1, 10)
    finally:
        ctl.stop()
