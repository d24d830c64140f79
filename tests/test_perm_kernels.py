"""Inner products and addDensityMatrix of registers whose qubits sit on
different positions (relabelling wave passes move each register's qubits its
own way): the permuted kernels read one register in the other's layout
(backend innerProductPerm / axpbyPerm) instead of relaying both out, as the
reference's local-sum-plus-allreduce needs no relayout either
(QuEST_cpu_distributed.c:41-51).  Checked against the NumPy oracle on the
wave planner's host emulation (QUEST_CPU_PLANNER=3) and on the GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import sys
import numpy as np
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi
from quest_amd.utils import oracle as O

n = int(sys.argv[1])
tol = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-11
env = qa.Env()
a, b = qa.Register(env, n), qa.Register(env, n)
oa = O.StateVector(n, np.full(1 << n, 1 / np.sqrt(1 << n)))
ob = O.StateVector(n, np.full(1 << n, 1 / np.sqrt(1 << n)))
a.init_plus()
b.init_plus()
ca, cb = random_layered(n, 8, seed=21), random_layered(n, 8, seed=22)
ca.apply(a); ca.apply_oracle(oa)
cb.apply(b); cb.apply_oracle(ob)
a.flush(); b.flush()
la, lb = capi.getQubitLayout(a.q), capi.getQubitLayout(b.q)
assert la != lb, (la, lb)   # different layouts, or the test checks nothing
capi.resetQuESTStats()
ip = a.inner(b)
want = np.vdot(oa.v, ob.v)
assert abs(ip - want) < tol, (ip, want)
st = capi.getQuESTStats()
assert st["permutedOps"] == 1 and st["relayouts"] == 0, st
# both layouts untouched by the inner product
assert capi.getQubitLayout(a.q) == la and capi.getQubitLayout(b.q) == lb
# addDensityMatrix: rho := (1 - p) rho + p sigma in rho's layout (axpbyPerm)
m = n // 2
rho, sig = qa.Register(env, m, density=True), qa.Register(env, m, density=True)
for reg, seed in ((rho, 31), (sig, 32)):
    reg.init_plus()
    random_layered(m, 8, seed=seed).apply(reg)
    reg.flush()
assert capi.getQubitLayout(rho.q) != capi.getQubitLayout(sig.q)
r2, s2 = qa.Register(env, m, density=True), qa.Register(env, m, density=True)
capi.cloneQureg(r2.q, rho.q)
capi.cloneQureg(s2.q, sig.q)
R, S = r2.to_numpy(), s2.to_numpy()   # canonicalises the copies only
capi.resetQuESTStats()
p = 0.3
capi.addDensityMatrix(rho.q, p, sig.q)
st = capi.getQuESTStats()
assert st["permutedOps"] == 1 and st["relayouts"] == 0, st
got = rho.to_numpy()
assert np.max(np.abs(got - ((1 - p) * R + p * S))) < tol
print("perm ok", ip)
'''


def _run(backend, n, extra=None, timeout=600, tol=1e-11):
    env = dict(os.environ, QUEST_BACKEND=backend, **(extra or {}))
    if backend == "cpu":
        env["QUEST_CPU_PLANNER"] = "3"
    out = subprocess.run([sys.executable, "-c", SCRIPT, str(n), repr(tol)], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "perm ok" in out.stdout


def test_permuted_kernels_emulated_on_host():
    _run("cpu", 20)


@pytest.mark.gpu
@pytest.mark.parametrize("prec,bits", [(2, 11), (2, 10), (2, 12), (1, 11)])
def test_permuted_kernels_gpu(prec, bits):
    """fp64 with 2^10 / 2^11 / 2^12-element tiles (2 / 4 / 8 element pairs a
    thread) and the fp32 library."""
    _run("hip", 22, extra={"QUEST_PREC": str(prec), "QUEST_PERM_TILE_BITS": str(bits)}, timeout=300,
         tol=1e-11 if prec == 2 else 2e-5)
