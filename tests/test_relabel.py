"""In-place relabelling passes (planTiles relabelFrom, src/core/tiles.cpp):
a wave pass may store its tile with the qubits permuted among the tile's
positions, so the register's logical->physical qubit map changes during a
flush.  Every read must still see the canonical state.  Runs on the host
emulation of the wave engine (QUEST_CPU_PLANNER=3, the same plans as the GPU)
in a subprocess, against the NumPy oracle; the GPU twin is in test_gpu.py."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, tempfile
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi
from quest_amd.utils import oracle as O

n = int(sys.argv[2])
env = qa.Env()
r = qa.Register(env, n)
r.init_plus()
o = O.StateVector(n, np.full(1 << n, 1 / np.sqrt(1 << n)))
c = random_layered(n, 10, seed=11)
capi.resetQuESTStats()
c.apply(r)
c.apply_oracle(o)
r.flush()
layout = capi.getQubitLayout(r.q)
moved = sum(1 for lg, p in enumerate(layout) if lg != p)
print("moved", moved, "passes", capi.getQuESTStats()["passes"])
relabel = capi.getQuESTTuning("wave_relabel")
assert relabel == 0 or moved > 0, layout
# single amplitudes and marginals in the permuted layout
rng = np.random.default_rng(3)
for i in rng.integers(0, 1 << n, 20):
    assert abs(r.amp(int(i)) - o.v[int(i)]) < 1e-12
for q in range(n):
    assert abs(r.prob(q, 1) - o.prob(q, 1)) < 1e-12
# a clone keeps the layout; inner products across layouts
b = qa.Register(env, n)
capi.cloneQureg(b.q, r.q)
assert abs(r.inner(b) - 1) < 1e-12
b.init_plus()
ip = r.inner(b)
assert abs(ip - np.vdot(o.v, np.full(1 << n, 1 / np.sqrt(1 << n)))) < 1e-12
# more gates after the relabelled flush, then a partial setAmps
c2 = random_layered(n, 4, seed=12)
c2.apply(r)
c2.apply_oracle(o)
vals = rng.normal(size=8) + 1j * rng.normal(size=8)
capi.setAmps(r.q, 100, vals.real.copy(), vals.imag.copy(), 8)
o.v[100:108] = vals
assert np.max(np.abs(r.to_numpy() - o.v)) < 1e-12
# checkpoint round trip after another relabelling flush
c3 = random_layered(n, 3, seed=13)
c3.apply(r)
c3.apply_oracle(o)
with tempfile.TemporaryDirectory() as d:
    path = os.path.join(d, "ck")
    assert capi.saveQuregCheckpoint(r.q, path)
    r2 = qa.Register(env, n)
    assert capi.loadQuregCheckpoint(r2.q, path)
    assert np.max(np.abs(r2.to_numpy() - o.v)) < 1e-12
print("relabel ok")
'''


@pytest.mark.parametrize("relabel", ["1", "0"])
def test_relabelled_layout_reads_match_oracle(relabel):
    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, "16"], cwd=ROOT, capture_output=True, text=True,
                         timeout=600, env=dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3",
                                               QUEST_WAVE_RELABEL=relabel))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "relabel ok" in out.stdout


def test_relabelling_cuts_passes():
    """The layered circuit needs fewer wave passes with relabelling."""
    code = ("import quest_amd as qa\n"
            "from quest_amd.models import random_layered\n"
            "e = qa.Env(); r = qa.Register(e, 18); r.init_plus(); qa.capi.resetQuESTStats()\n"
            "random_layered(18, 16, seed=7).apply(r); r.sync()\n"
            "print('passes', qa.capi.getQuESTStats()['passes'])\n")
    res = {}
    for relabel in ("0", "1"):
        out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3",
                                      QUEST_WAVE_RELABEL=relabel))
        assert out.returncode == 0, out.stderr[-2000:]
        res[relabel] = int(out.stdout.split()[-1])
    assert res["1"] < res["0"], res


DENSITY = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import quest_amd as qa
from helpers import apply_random_ops, oracle_for
from quest_amd.ops import capi

env = qa.Env()
n = 7                      # 14 state-vector qubits: wave passes on the host emulation
r = qa.Register(env, n, density=True)
rng = np.random.default_rng(5)
o = oracle_for(r, rng)
apply_random_ops(r, o, rng, 120)          # gates only: the flushes relabel
r.flush()
moved = sum(1 for lg, p in enumerate(capi.getQubitLayout(r.q)) if lg != p)
print("moved", moved)
assert moved > 0
assert np.max(np.abs(r.to_numpy() - o.rho)) < 1e-11
assert abs(r.purity() - o.purity()) < 1e-11
assert abs(r.total_prob() - np.real(np.trace(o.rho))) < 1e-11
for q in range(n):
    assert abs(r.prob(q, 0) - o.prob(q, 0)) < 1e-11
for (i, j) in [(0, 0), (3, 5), (127, 64)]:
    a = capi.getDensityAmp(r.q, i, j)
    assert abs(complex(a.real, a.imag) - o.rho[i, j]) < 1e-11
psi = qa.Register(env, n)
psi.init_plus()
f = capi.calcFidelity(r.q, psi.q)
v = np.full(1 << n, 1 / np.sqrt(1 << n))
assert abs(f - np.real(np.conj(v) @ o.rho @ v)) < 1e-11
print("density relabel ok")
'''


def test_relabelled_density_matrix_reads():
    out = subprocess.run([sys.executable, "-c", DENSITY, ROOT], cwd=ROOT, capture_output=True, text=True,
                         timeout=600, env=dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3"))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "density relabel ok" in out.stdout
