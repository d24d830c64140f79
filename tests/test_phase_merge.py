"""Phase ops on the same amplitudes inside a run of diagonal ops are merged
by the wave lowering (mergePhases in src/core/wave.cpp: Z Z, T T -> S, the
CZ pairs the conditional frame puts around consecutive rotations of a
conditioned target, ...).  A circuit built to produce such runs, on the
wave planner's host emulation and on the GPU, against the NumPy oracle;
merging must remove wave ops and change nothing else."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import math
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
from quest_amd.utils import oracle as O

import sys
n = int(sys.argv[1])
e = qa.Env()
r = qa.Register(e, n)
rng = np.random.default_rng(11)
psi = O.random_state(rng, n)
r.set_amps(psi)
o = O.StateVector(n, psi.copy())
r.sync()
capi.resetQuESTStats()
CZ = np.diag([1, 1, 1, -1])
for layer in range(6):
    for q in range(0, n, 3):
        # runs of phases on one qubit (Z Z, T T, S Z, Rz Rz)
        r.z(q); o.apply(O.Z, q)
        r.t(q); o.apply(O.T, q)
        r.t(q); o.apply(O.T, q)
        r.rz(q, 0.3 + layer); o.apply(O.rot(0.3 + layer, (0, 0, 1)), q)
        r.z(q); o.apply(O.Z, q)
        r.rz(q, -0.1); o.apply(O.rot(-0.1, (0, 0, 1)), q)
    for q in range(0, n - 1, 2):
        # a CNOT (deferred by the conditional frame) then rotations of its target
        r.cnot(q, q + 1); o.apply(O.X, q + 1, [q])
        r.ry(q + 1, 0.4); o.apply(O.rot(0.4, (0, 1, 0)), q + 1)
        r.ry(q + 1, -0.7); o.apply(O.rot(-0.7, (0, 1, 0)), q + 1)
        r.cz(q, q + 1); o.apply(CZ, [q, q + 1])
        r.cz(q, q + 1); o.apply(CZ, [q, q + 1])
        r.s(q); o.apply(O.S, q)
        r.s(q); o.apply(O.S, q)
    for q in range(1, n, 4):
        r.h(q); o.apply(O.H, q)
        r.rx(q, 0.2 * layer); o.apply(O.rot(0.2 * layer, (1, 0, 0)), q)
r.sync()
st = capi.getQuESTStats()
got = r.to_numpy()
err = np.max(np.abs(got - o.v))
print("MERGE err %.3e waveOps %d passes %d" % (err, st["waveOps"], st["passes"]))
assert err < TOL, err
assert st["wavePasses"] >= 1, st
'''


def _run(backend, merge, tol, n, **knobs):
    env = dict(os.environ, QUEST_BACKEND=backend, QUEST_WAVE_MERGE_PHASES=merge, **knobs)
    if backend == "cpu":
        env["QUEST_CPU_PLANNER"] = "3"
    out = subprocess.run([sys.executable, "-c", SCRIPT.replace("TOL", repr(tol)), str(n)], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("MERGE")][0]
    f = line.split()
    return int(f[4]), int(f[6])


def _check(backend, tol, n):
    ops_on, passes_on = _run(backend, "1", tol, n)
    ops_off, passes_off = _run(backend, "0", tol, n)
    assert passes_on == passes_off   # the lowering, not the plan, changes
    assert ops_on < ops_off, (ops_on, ops_off)


def test_phase_merge_on_the_wave_emulation():
    _check("cpu", 1e-12, 16)


@pytest.mark.gpu
def test_phase_merge_gpu():
    _check("hip", 1e-12, 20)   # the GPU takes the wave engine from 19 local qubits


def _check_frame(backend, tol, n):
    """The phase frame (zFrame in src/core/wave.cpp): single-location phases
    carried along the pass and merged per location, signs absorbed by the 2x2
    ops and CNOTs after them.  Same plans, fewer wave ops, the oracle's state."""
    ops_p, passes_p = _run(backend, "1", tol, n)
    ops_z, passes_z = _run(backend, "1", tol, n, QUEST_WAVE_PFRAME="0")
    ops_0, passes_0 = _run(backend, "1", tol, n, QUEST_WAVE_ZFRAME="0")
    assert passes_p == passes_z == passes_0
    assert ops_p < ops_z <= ops_0, (ops_p, ops_z, ops_0)


def test_phase_frame_on_the_wave_emulation():
    _check_frame("cpu", 1e-12, 16)


@pytest.mark.gpu
def test_phase_frame_gpu():
    _check_frame("hip", 1e-12, 20)
