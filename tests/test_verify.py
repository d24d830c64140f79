"""Debug verify mode (QUEST_VERIFY=1 / tuning "verify"): every fused flush is
re-executed op by op on a shadow copy of the state and compared, the
"run every kernel against a reference" debug mode of SURVEY.md §5.2.  The
detector itself is tested by injecting a one-off corruption into a verified
flush ("verify_inject"), which must end the process with a report."""
import math
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_INJECT = r"""
import quest_amd as qa
from quest_amd.ops import capi
env = qa.Env()
reg = qa.Register(env, {n})
capi.setQuESTTuning("verify", 1)
for q in range({n}):
    reg.h(q)
reg.sync()
assert capi.getQuESTStats()["verifiedFlushes"] >= 1
capi.setQuESTTuning("verify_inject", 1)
for q in range({n}):
    reg.rx(q, 0.3)
reg.sync()
print("NOT DETECTED")
"""


def _verified_random_circuit(env, n, depth, seed):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi
    from quest_amd.utils import oracle as O

    capi.resetQuESTStats()
    assert capi.setQuESTTuning("verify", 1) == 1
    try:
        c = random_layered(n, depth, seed=seed)
        reg = qa.Register(env, n)
        reg.init_plus()
        c.apply(reg)
        got = reg.to_numpy()
        reg.close()
    finally:
        capi.setQuESTTuning("verify", 0)
    st = capi.getQuESTStats()
    o = O.StateVector(n, np.full(1 << n, 1 / math.sqrt(1 << n)))
    c.apply_oracle(o)
    assert np.max(np.abs(got - o.v)) < 1e-10
    return st


def _inject(backend, n):
    envv = dict(os.environ, QUEST_BACKEND=backend)
    out = subprocess.run([sys.executable, "-c", _INJECT.format(n=n)], cwd=ROOT, env=envv, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode != 0, out.stdout
    assert "NOT DETECTED" not in out.stdout
    assert "QuEST verify" in out.stderr and "differs from op-by-op" in out.stderr, out.stderr[-2000:]


def test_verify_mode_checks_every_flush(env):
    st = _verified_random_circuit(env, 14, 8, seed=5)
    assert st["verifiedFlushes"] >= 1
    # the shadow run is not counted as work
    assert st["passes"] < 8 * 21


def test_verify_detects_injected_fault():
    _inject("cpu", 12)


@pytest.mark.gpu
def test_verify_mode_on_gpu():
    import quest_amd as qa

    e = qa.Env()
    assert qa.capi.getQuESTBackend() == "HIP"
    st = _verified_random_circuit(e, 22, 10, seed=9)
    assert st["verifiedFlushes"] >= 1


@pytest.mark.gpu
def test_verify_detects_injected_fault_on_gpu():
    _inject("hip", 20)
