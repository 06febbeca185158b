import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    # The product uses camera-ray tile lists only for shares with >= 6 items per resident lane
    # (rt_render); the parity tests' small images would never reach them, so every Context the tests
    # create forces them on (test_camera_lists_on_and_off covers the default threshold).
    import raytracing_gpu_amd as rt

    rt.DEFAULT_OPTIONS["bins_min_items_per_lane"] = 0.0


@pytest.fixture(scope="session")
def oracle():
    """The CPU oracle (test infrastructure); built in-tree if absent."""
    from oracle import ref_cpu

    if not os.path.exists(ref_cpu.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    return ref_cpu


@pytest.fixture(scope="session")
def rtlib():
    import raytracing_gpu_amd as rt

    rt.lib()  # raises when librt_hip.so is missing: no fallback
    return rt


@pytest.fixture(scope="session")
def gpu_ctx(rtlib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = rtlib.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture
def ctx_opts(gpu_ctx):
    """Set rt_ctx_options on the session context for one test (include/rt_hip.h); the options are
    restored afterwards.  Upload-time options take effect at the test's next upload."""
    before = gpu_ctx.options()
    yield lambda **kw: gpu_ctx.set_options(**kw)
    gpu_ctx.set_options(**before)
