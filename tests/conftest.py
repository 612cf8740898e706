import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # test infrastructure: the CPU checker
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))  # variant_specs (fixture specs)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 device (run on the MI355X box)")


@pytest.fixture(scope="session")
def cfg():
    from sdf_nmpc_amd.config import Config
    return Config()


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    return {k: np.load(os.path.join(d, f"{k}_golden.npz")) for k in ("sdf", "lin", "grid", "params", "sdfc3",
                                                                                  "variants", "scene")}


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test on a machine without a HIP device")
    from sdf_nmpc_amd import _lib
    ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)  # ordered with torch's stream
    yield ctx
    ctx.close()
