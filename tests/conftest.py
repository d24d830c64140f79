"""pytest configuration.

* ``gpu`` marker: test needs a real MI355X (run with ``-m gpu``; the HIP
  library is used).  Everything else runs on CPU with the host build.
* The backend is chosen once per session from the marker expression, because
  a process binds one native library (QUEST_BACKEND overrides).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (HIP backend)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    markexpr = (config.getoption("-m") or "").strip()
    if "QUEST_BACKEND" not in os.environ:
        os.environ["QUEST_BACKEND"] = "hip" if markexpr == "gpu" else "cpu"
    _ensure_built(os.environ["QUEST_BACKEND"])


def _ensure_built(backend):
    import glob

    lib = os.path.join(ROOT, "quest_amd", "lib", f"libQuEST_{backend}_f64.so")
    fast = glob.glob(os.path.join(ROOT, "quest_amd", "ops", "_gatecall*.so"))
    if not os.path.exists(lib) or not fast:
        import subprocess

        subprocess.run(["make", "-C", ROOT, "-j8", backend], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def env():
    import quest_amd as qa

    return qa.Env()


@pytest.fixture
def rng():
    import numpy as np

    return np.random.default_rng(1234)
