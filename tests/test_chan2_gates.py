"""Two-qubit density channels lowered to one-qubit ops (src/api/api.cpp
twoQubitChannelsAsGates): 2q depolarising (every build) and 2q dephasing
(fp32, and fp64 below the diagonal-form threshold) in the "differs" frame
-- CNOTs c ^= r, deferred Xs, a diagonal on the coherences and controlled real
2x2 mixes of the populations (the reference's delta / gamma three-step form,
QuEST_cpu_local.c:40-51).  Against the Kraus-operator oracle, through the
wave planner's host emulation at wave size, and the channel fallback."""
import os
import subprocess
import sys

import numpy as np
import pytest

import quest_amd as qa
from helpers import assert_close, oracle_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P2 = [0.0, 1e-6, 0.05, 0.3, 0.6, 0.9, 15 / 16]


@pytest.mark.parametrize("p", P2)
def test_two_qubit_depolarise_vs_oracle(env, p):
    rng = np.random.default_rng(int(p * 1e6) + 7)
    reg = qa.Register(env, 4, density=True)
    o = oracle_for(reg, rng)
    for a, b in ((0, 1), (3, 1), (2, 0), (1, 3)):
        reg.depolarise2(a, b, p)
        o.depolarise2(a, b, p)
        reg.ry(a, 0.3)
        o.apply(np.array([[np.cos(0.15), -np.sin(0.15)], [np.sin(0.15), np.cos(0.15)]]), a)
    assert_close(reg, o, 1e-12)
    assert abs(reg.total_prob() - np.real(np.trace(o.rho))) < 1e-12
    assert abs(reg.purity() - o.purity()) < 1e-12
    reg.close()


def test_strong_two_qubit_dephase_vs_oracle(env):
    """Factors below the diagonal form's threshold take the gate form."""
    rng = np.random.default_rng(11)
    reg = qa.Register(env, 4, density=True)
    o = oracle_for(reg, rng)
    for a, b, p in ((0, 1, 0.7499), (2, 3, 0.75), (1, 2, 0.74995)):
        reg.dephase2(a, b, p)
        o.dephase2(a, b, p)
    assert_close(reg, o, 1e-12)
    reg.close()


WAVE = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1] + "/tests")
import quest_amd as qa
from helpers import apply_random_ops, assert_close, oracle_for
from quest_amd.ops import capi
env = qa.Env()
rng = np.random.default_rng(5)
n = 10    # 20-qubit state: wave passes on the host planner (the HIP backend's threshold: L >= 19)
reg = qa.Register(env, n, density=True)
o = oracle_for(reg, rng)
capi.resetQuESTStats()
for step in range(4):
    apply_random_ops(reg, o, rng, 12)
    for a, b in ((0, 1), (2, 5), (9, 3)):
        p = float(rng.uniform(0, 15 / 16))
        reg.depolarise2(a, b, p)
        o.depolarise2(a, b, p)
        p = float(rng.uniform(0, 0.75))
        reg.dephase2(b, a, p)
        o.dephase2(b, a, p)
reg.sync()
st = capi.getQuESTStats()   # before reading the state back (which restores the canonical layout)
print("passes", st["passes"], "wave", st["wavePasses"])
assert st["wavePasses"] == st["passes"], st
assert_close(reg, o, 1e-11)
'''


def test_two_qubit_channels_on_the_wave_planner():
    """A 10-qubit density matrix (20-qubit state) under gates and 2q channels:
    every pass is a wave pass (host emulation of the GPU plans)."""
    env = dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3")
    out = subprocess.run([sys.executable, "-c", WAVE, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]


FP32 = r'''
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
from quest_amd.utils import oracle as O
assert capi.getQuEST_PREC() == 1
e = qa.Env()
r = qa.Register(e, 4, density=True)
rng = np.random.default_rng(3)
rho = O.random_density(rng, 4)
r.set_amps(rho.flatten(order="F"))
o = O.DensityMatrix(4, rho.copy())
for a, b, p in ((0, 1, 0.3), (2, 3, 0.7), (1, 2, 0.5)):
    r.depolarise2(a, b, p); o.depolarise2(a, b, p)
    r.dephase2(a, b, p / 2); o.dephase2(a, b, p / 2)
got = r.to_numpy().reshape(16, 16, order="F")
err = np.max(np.abs(got - o.rho))
print("fp32 err", err)
assert err < 1e-6, err
'''


def test_fp32_two_qubit_channels():
    env = dict(os.environ, QUEST_PREC="1", QUEST_BACKEND=os.environ.get("QUEST_BACKEND", "cpu"))
    out = subprocess.run([sys.executable, "-c", FP32], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]


FALLBACK = r'''
import numpy as np, sys
sys.path.insert(0, sys.argv[1] + "/tests")
import quest_amd as qa
from helpers import assert_close, oracle_for
e = qa.Env()
rng = np.random.default_rng(9)
r = qa.Register(e, 4, density=True)
o = oracle_for(r, rng)
for a, b, p in ((0, 1, 0.3), (3, 2, 0.9)):
    r.depolarise2(a, b, p); o.depolarise2(a, b, p)
    r.dephase2(a, b, 0.7499); o.dephase2(a, b, 0.7499)
assert_close(r, o, 1e-12)
'''


def test_channel_op_fallback():
    """QUEST_CHAN2_GATES=0 keeps the 16-element channel op."""
    env = dict(os.environ, QUEST_CHAN2_GATES="0", QUEST_BACKEND=os.environ.get("QUEST_BACKEND", "cpu"))
    out = subprocess.run([sys.executable, "-c", FALLBACK, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]


CHAN_RELABEL = r'''
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
from quest_amd.utils import oracle as O
n = 10
e = qa.Env()
r = qa.Register(e, n, density=True)
rng = np.random.default_rng(12)
rho = O.random_density(rng, n)
r.set_amps(rho.flatten(order="F"))
o = O.DensityMatrix(n, rho.copy())
H = np.array([[1, 1], [1, -1]]) / np.sqrt(2)
for rep in range(2):
    for q in range(n):
        r.damping(q, 0.1 + 0.02 * q); o.damping(q, 0.1 + 0.02 * q)
    for q in range(0, n, 3):
        r.h(q); o.apply(H, q)
    for q in range(n):
        r.depolarise(q, 0.05); o.depolarise(q, 0.05)
r.sync()
st = capi.getQuESTStats()
got = r.to_numpy().reshape(1 << n, 1 << n, order="F")
err = np.max(np.abs(got - o.rho))
print("chan relabel err", err, "passes", st["passes"], "wave", st["wavePasses"])
assert err < 1e-12, err
'''


@pytest.mark.parametrize("relabel,cmin", [("1", "4"), ("1", "5"), ("0", "4")])
def test_channel_flush_relabelling(relabel, cmin):
    """One-qubit damping / depolarising (register channels CH1 on row and
    column bits) in flushes that relabel (QUEST_WAVE_CHAN_RELABEL=1) and keep
    fewer always-resident positions (QUEST_WAVE_CMIN_CHAN), on the wave
    planner's host emulation against the Kraus oracle."""
    env = dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3", QUEST_WAVE_CHAN_RELABEL=relabel,
               QUEST_WAVE_CMIN_CHAN=cmin)
    out = subprocess.run([sys.executable, "-c", CHAN_RELABEL], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "chan relabel err" in out.stdout
