"""The Python binding's per-gate fast path (src/py/gatecall.c): a Register's
one- and two-qubit gate methods call the exported C functions through the
CPython C API instead of ctypes.  Same functions, so the same state, the same
validation errors (QuESTError with the reference's codes), the same QASM; in
every precision the library is built for (the angle's C type follows
QuEST_PREC)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import quest_amd as qa
from quest_amd.models import random_mixed
from quest_amd.ops import capi
from quest_amd.ops.capi import QuESTError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SLOW = {"h": "hadamard", "x": "pauliX", "y": "pauliY", "z": "pauliZ", "s": "sGate", "t": "tGate",
        "rx": "rotateX", "ry": "rotateY", "rz": "rotateZ", "phase": "phaseShift", "cnot": "controlledNot",
        "cy": "controlledPauliY", "cz": "controlledPhaseFlip", "crx": "controlledRotateX",
        "cry": "controlledRotateY", "crz": "controlledRotateZ", "cphase": "controlledPhaseShift"}


def _apply_slow(reg, circ):
    """The same gates through the ctypes wrappers (capi.<C name>)."""
    for g in circ.gates:
        if g.name == "mcz":
            reg.mcz(list(g.qubits))
            continue
        args = list(g.qubits) + ([] if g.param is None else [g.param])
        getattr(capi, SLOW[g.name])(reg.q, *args)


def test_fast_path_is_bound(env):
    r = qa.Register(env, 3)
    try:
        assert capi.binding().gatecall() is not None, "src/py/gatecall.c not built (make cpu)"
        assert type(r.h).__name__ == "builtin_function_or_method"
        assert type(r.crz).__name__ == "builtin_function_or_method"
    finally:
        r.close()


@pytest.mark.parametrize("density", [False, True])
def test_fast_path_matches_ctypes_path(env, density):
    n = 5 if density else 9
    circ = random_mixed(n, 300, seed=3)
    a = qa.Register(env, n, density=density)
    b = qa.Register(env, n, density=density)
    try:
        a.init_plus()
        b.init_plus()
        circ.apply(a)
        _apply_slow(b, circ)
        np.testing.assert_array_equal(a.to_numpy(), b.to_numpy())
    finally:
        a.close()
        b.close()


def test_fast_path_errors_and_arguments(env):
    r = qa.Register(env, 4)
    try:
        r.init_zero()
        with pytest.raises(QuESTError) as ei:
            r.h(4)
        assert ei.value.function == "hadamard" and ei.value.code != 0
        with pytest.raises(QuESTError) as ei:
            r.cnot(2, 2)
        assert ei.value.function == "controlledNot"
        with pytest.raises(QuESTError):
            r.crz(-1, 0, 0.5)
        with pytest.raises(QuESTError):
            r.rx(2 ** 40, 0.1)      # outside C int: rejected, not wrapped
        # after the errors the register works and nothing is left pending
        assert capi.binding().nerr == 0
        r.x(np.int64(1))            # numpy scalars as arguments
        r.ry(0, np.float32(0.25))
        r.rz(0, 1)                  # an int angle
        ref = qa.Register(env, 4)
        try:
            ref.init_zero()
            capi.pauliX(ref.q, 1)
            capi.rotateY(ref.q, 0, 0.25)
            capi.rotateZ(ref.q, 0, 1.0)
            np.testing.assert_array_equal(r.to_numpy(), ref.to_numpy())
        finally:
            ref.close()
        with pytest.raises(TypeError):
            r.h(0, 1)
        with pytest.raises(TypeError):
            r.rx(0, "a")
    finally:
        r.close()
    # a closed register's methods are the class's again (ctypes path)
    assert "h" not in vars(r)


def test_fast_path_records_qasm(env):
    a = qa.Register(env, 3)
    b = qa.Register(env, 3)
    try:
        for reg, fast in ((a, True), (b, False)):
            reg.start_qasm()
            if fast:
                reg.h(0), reg.cnot(0, 1), reg.crz(1, 2, 0.125), reg.phase(2, 0.5), reg.cz(0, 2)
            else:
                capi.hadamard(reg.q, 0), capi.controlledNot(reg.q, 0, 1)
                capi.controlledRotateZ(reg.q, 1, 2, 0.125), capi.phaseShift(reg.q, 2, 0.5)
                capi.controlledPhaseFlip(reg.q, 0, 2)
        assert a.qasm == b.qasm
        assert len(a.qasm.strip().splitlines()) >= 5
    finally:
        a.close()
        b.close()


CHILD = r'''
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
from quest_amd.models import random_mixed
assert capi.binding().gatecall() is not None
e = qa.Env()
circ = random_mixed(6, 200, seed=5)
a, b = qa.Register(e, 6), qa.Register(e, 6)
a.init_plus(); b.init_plus()
circ.apply(a)
import test_gatecall as T
T._apply_slow(b, circ)
assert np.array_equal(a.to_numpy(), b.to_numpy())
print("ok", capi.getQuEST_PREC())
'''


@pytest.mark.parametrize("prec", ["1", "4"])
def test_fast_path_other_precisions(prec):
    env = dict(os.environ, QUEST_PREC=prec, QUEST_BACKEND="cpu",
               PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]))
    p = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert p.stdout.split()[-1] == prec
