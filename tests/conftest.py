import os
import sys

# CPU runs: engines, gloo ranks and reference ops each start an OpenMP pool; with
# one pool per process sized to every core, multi-process tests oversubscribe the
# CPUs and spin-waiting pools slow them ~10x. An explicit setting (the GPU box
# exports 16) wins.
os.environ.setdefault("OMP_NUM_THREADS", "2")

import pytest  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _seed_torch():
    """This PyTorch build seeds its default generator randomly per process, and
    many tests build random-init tiny models whose greedy outputs are compared
    across parallel layouts (TP / EP / DBO sum in other orders): a fixed seed
    keeps those models - and any near-ties in their logits - the same every run."""
    import torch

    torch.manual_seed(int(os.environ.get("LLMD_TEST_SEED", "0")))
    yield
