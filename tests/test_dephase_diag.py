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


FOLD = r'''
import sys
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
from quest_amd.utils import oracle as O
n = 10
e = qa.Env()
r = qa.Register(e, n, density=True)
rng = np.random.default_rng(5)
psi = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
psi /= np.linalg.norm(psi)
rho = np.outer(psi, psi.conj())
r.set_amps(rho.flatten(order="F"))
o = O.DensityMatrix(n, rho.copy())
r.sync()
capi.resetQuESTStats()
for a in range(0, n - 1, 2):
    r.dephase2(a, a + 1, 0.3); o.dephase2(a, a + 1, 0.3)
for q in (1, 4, 8):
    r.dephase(q, 0.2); o.dephase(q, 0.2)
r.h(3); o.apply(np.array([[1, 1], [1, -1]]) / np.sqrt(2), 3)
for a in range(1, n - 1, 2):
    r.dephase2(a, a + 1, 0.45); o.dephase2(a, a + 1, 0.45)
r.sync()
st = capi.getQuESTStats()
got = r.to_numpy().reshape(1 << n, 1 << n, order="F")
err = np.max(np.abs(got - o.rho))
print("fold err", err, "passes", st["passes"], "wave", st["wavePasses"], "waveOps", st["waveOps"])
assert err < 1e-12, err
assert st["wavePasses"] == st["passes"] >= 1, st
'''


@pytest.mark.parametrize("fold", ["1", "0"])
def test_folded_diagonal_runs_on_the_wave_planner(fold):
    """Runs of dephasing factors (diagonal ops whose masks lie partly or wholly
    outside the tile) folded per in-tile mask into one op per value of their
    outside bits (ctrlOut / ctrlOutZero), on the wave planner's host emulation
    of a 10-qubit density matrix, against the Kraus oracle;
    QUEST_WAVE_FOLD_DIAG=0 emits every op."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3", QUEST_WAVE_FOLD_DIAG=fold)
    out = subprocess.run([sys.executable, "-c", FOLD], cwd=root, env=env, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "fold err" in out.stdout


@pytest.mark.gpu
def test_folded_diagonal_runs_gpu():
    """The same on the GPU kernel (check path with out-of-tile zero bits)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = FOLD.replace("n = 10", "n = 11")
    env = dict(os.environ, QUEST_BACKEND="hip")
    out = subprocess.run([sys.executable, "-c", script], cwd=root, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "fold err" in out.stdout
