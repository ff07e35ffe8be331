"""EPP metrics batch Counter/Histogram children (router/metrics.py _Deferred):
the exposition must equal what per-call prometheus observe/inc would give."""
import random

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

from llmd_amd.router.metrics import SMALL, EPPMetrics


def _samples(text: bytes, family: str) -> dict:
    out = {}
    for line in text.decode().splitlines():
        if line.startswith(family) and not line.startswith("#") and "_created" not in line:
            k, v = line.rsplit(" ", 1)
            out[k] = float(v)
    return out


def test_deferred_histogram_and_counter_match_prometheus():
    m = EPPMetrics()
    reg = CollectorRegistry()
    h = Histogram("inference_extension_plugin_duration_seconds", "Plugin latency",
                  ["extension_point", "plugin_type", "plugin_name"], buckets=SMALL, registry=reg)
    c = Counter("inference_objective_request", "Requests", ["model_name", "target_model_name", "priority"],
                registry=reg)
    rnd = random.Random(0)
    # bucket bounds exactly, values between, beyond the last bound, and more than one flush batch
    vals = list(SMALL) + [rnd.random() * 0.02 for _ in range(5000)] + [1e4, 0.0]
    for v in vals:
        m.child(m.plugin_dur, "Scorer", "queue-scorer", "q").observe(v)
        h.labels("Scorer", "queue-scorer", "q").observe(v)
    for i in range(3000):
        m.child(m.req_total, "m", "m", "0").inc()
        c.labels("m", "m", "0").inc()
    mine = _samples(m.render(), "inference_extension_plugin_duration_seconds")
    ref = _samples(generate_latest(reg), "inference_extension_plugin_duration_seconds")
    assert mine.keys() == ref.keys() and mine
    for k in ref:
        assert abs(mine[k] - ref[k]) <= 1e-9 * max(1.0, abs(ref[k])), k
    assert _samples(m.render(), "inference_objective_request_total") == \
        _samples(generate_latest(reg), "inference_objective_request_total")
    # a second render without new observations is unchanged (nothing counted twice)
    assert _samples(m.render(), "inference_extension_plugin_duration_seconds") == mine


def test_engine_batched_itl_ttft_exposed_on_scrape():
    from llmd_amd.engine.request import SamplingParams
    from tests.test_engine import make_engine

    eng = make_engine()
    for i, n in enumerate((5, 9, 14)):
        eng.add_request(f"r{i}", list(range(3, 3 + n)), SamplingParams(max_tokens=5, temperature=0.0,
                                                                      ignore_eos=True))
    while eng.has_unfinished():
        eng.step()
    text = eng.metrics.render().decode()

    def count(name):
        return sum(float(ln.rsplit(" ", 1)[1]) for ln in text.splitlines() if ln.startswith(name + "_count"))

    assert count("vllm:inter_token_latency_seconds") == len(eng.metrics.itls) > 0
    assert count("vllm:time_to_first_token_seconds") == len(eng.metrics.ttfts) == 3


def test_concurrent_flush_and_observe_is_exact():
    """the engine thread's 4096-item flush and a scrape's flush can
    run at once; neither may raise and no observation may be lost."""
    import threading

    from llmd_amd.utils.prom import Deferred

    reg = CollectorRegistry()
    h = Histogram("t_h", "h", registry=reg, buckets=(1.0, 2.0, 4.0))
    d = Deferred(h)
    errors = []
    n_per, n_thr = 20000, 3

    def produce():
        try:
            for i in range(n_per):
                d.observe(float(i % 5))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def scrape(stop):
        try:
            while not stop.is_set():
                d.flush()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    stop = threading.Event()
    scr = [threading.Thread(target=scrape, args=(stop,)) for _ in range(2)]
    prod = [threading.Thread(target=produce) for _ in range(n_thr)]
    for t in scr + prod:
        t.start()
    for t in prod:
        t.join()
    stop.set()
    for t in scr:
        t.join()
    d.flush()
    assert not errors, errors
    total = sum(b.get() for b in h._buckets)
    assert total == n_per * n_thr
