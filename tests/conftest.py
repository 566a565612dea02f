import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT,):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built engine")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def fold1():
    z = np.load(os.path.join(GOLDEN, "ml100k_fold1.npz"))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def streams():
    z = np.load(os.path.join(GOLDEN, "sampler_streams.npz"))
    return {k: z[k] for k in z.files}


def get_stream(streams, name):
    out = {"pairs": streams[name + "/pairs"], "negs": streams[name + "/negs"]}
    if name + "/groups" in streams:
        out["groups"] = streams[name + "/groups"]
    return out


@pytest.fixture(scope="session")
def gpu_available():
    try:
        from collaborativefilteringusingtensorflow_amd import _native as N
        return N.device_count() > 0
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _require_gpu(request):
    if request.node.get_closest_marker("gpu") is not None:
        from collaborativefilteringusingtensorflow_amd import _native as N
        # fail loudly (not skip) when the native library is missing on a GPU run
        N.lib()
        if N.device_count() == 0:
            pytest.skip("no HIP device visible")
