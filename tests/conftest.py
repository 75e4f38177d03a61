import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP C-ABI)")


@pytest.fixture(scope="session")
def blob():
    from mujoco_playground_amd import _lib
    return _lib.load_blob()


@pytest.fixture(scope="session")
def oracle(blob):
    from oracle.oracle import Oracle
    return Oracle(blob)


@pytest.fixture(scope="session")
def cmodel():
    """Compiled model (needs the reference MJCF; only in the build container)."""
    from mujoco_playground_amd.model.compiler import compile_mjcf, default_model_path
    p = default_model_path()
    if not os.path.exists(p):
        pytest.skip("reference MJCF not present")
    return compile_mjcf(p)


def f64_state(st_soa):
    """[44, N] float32 device/host tensor (uint32 words 42/43) -> [N, 44] float64."""
    s = st_soa.detach().cpu().numpy().T.copy() if hasattr(st_soa, "detach") else st_soa.T.copy()
    out = s.astype(np.float64)
    out[:, 42] = s[:, 42].view(np.uint32)
    out[:, 43] = s[:, 43].view(np.uint32)
    return out
