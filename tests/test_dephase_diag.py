"""Dephasing channels lowered to diagonal ops (src/api/api.cpp
applyOneQubitDephaseError / applyTwoQubitDephaseError): the factor on the
elements whose row and column bits differ is split into factors on all-ones
masks, so the channel needs no tile bits.  Strengths at the edge of the range
(factor 0, factor just above the 1e-3 switch-over) and the channel fallback
are compared with the Kraus-operator oracle.  Reference semantics:
QuEST.c mixDephasing / mixTwoQubitDephasing."""
import numpy as np
import pytest

import quest_amd as qa
from helpers import assert_close, oracle_for

P1 = [0.0, 0.1, 0.3, 0.4994, 0.4996, 0.5]          # factor 1 - 2p: 1 ... 0.0012, 0.0008, 0
P2 = [0.0, 0.2, 0.5, 0.74915, 0.74935, 0.75]       # factor 1 - 4p/3: 1 ... 0.00113, 0.00087, 0


@pytest.mark.parametrize("p", P1)
def test_one_qubit_dephase_vs_oracle(env, p):
    rng = np.random.default_rng(int(p * 1e4))
    reg = qa.Register(env, 4, density=True)
    o = oracle_for(reg, rng)
    for q in (0, 2, 3):
        reg.dephase(q, p)
        o.dephase(q, p)
    reg.h(1)
    o.apply(np.array([[1, 1], [1, -1]]) / np.sqrt(2), 1)
    reg.dephase(1, p)
    o.dephase(1, p)
    assert_close(reg, o, 1e-12)
    reg.close()


@pytest.mark.parametrize("p", P2)
def test_two_qubit_dephase_vs_oracle(env, p):
    rng = np.random.default_rng(int(p * 1e5) + 1)
    reg = qa.Register(env, 4, density=True)
    o = oracle_for(reg, rng)
    for a, b in ((0, 1), (3, 1), (2, 0)):
        reg.dephase2(a, b, p)
        o.dephase2(a, b, p)
    assert_close(reg, o, 1e-12)
    assert abs(reg.total_prob() - 1) < 1e-12
    reg.close()


def test_dephase_fuses_into_one_pass(env):
    """A run of dephasings on every qubit is diagonal: one fused pass."""
    from quest_amd.ops import capi

    reg = qa.Register(env, 6, density=True)
    reg.init_plus()
    reg.sync()
    capi.resetQuESTStats()
    for q in range(6):
        reg.dephase(q, 0.1)
    for q in range(5):
        reg.dephase2(q, q + 1, 0.1)
    reg.sync()
    assert capi.getQuESTStats()["passes"] == 1
    reg.close()


FP32_POPS = r'''
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
assert capi.getQuEST_PREC() == 1
e = qa.Env()
r = qa.Register(e, 5, density=True)
r.init_plus()
for q in range(5):
    r.h(q); r.ry(q, 0.3 * (q + 1))
r.sync()
before = r.to_numpy().reshape(32, 32, order="F")
for q in range(5):
    r.dephase(q, 0.37)
for q in range(4):
    r.dephase2(q, q + 1, 0.61)
after = r.to_numpy().reshape(32, 32, order="F")
d0, d1 = np.diag(before), np.diag(after)
print("pops", np.max(np.abs(d1 - d0)), "trace", abs(np.trace(after) - np.trace(before)))
assert np.array_equal(d0, d1), np.max(np.abs(d1 - d0))
'''


def test_fp32_dephasing_leaves_populations_untouched():
    """fp32 keeps the channel forms: the populations (diagonal of
    rho) come out bit for bit unchanged, as in the reference's kernels."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QUEST_PREC="1", QUEST_BACKEND=os.environ.get("QUEST_BACKEND", "cpu"))
    out = subprocess.run([sys.executable, "-c", FP32_POPS], cwd=root, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
