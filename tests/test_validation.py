"""Input validation: every reference error code (QuEST_validation.c:19-80)
is raised by the API calls that the reference validates, with the same
message; a rejected call leaves the state untouched; without a handler the
library prints the reference's banner and exits with the code."""
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from quest_amd.ops import capi
from quest_amd.ops.capi import QuESTError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

I2 = [[1, 0], [0, 1]]


@pytest.fixture
def regs(env):
    e = env.env
    r = {
        "q": capi.createQureg(3, e),
        "q4": capi.createQureg(4, e),
        "q6": capi.createQureg(6, e),
        "d": capi.createDensityQureg(3, e),
        "d2": capi.createDensityQureg(3, e),
    }
    yield r, e
    for q in r.values():
        capi.destroyQureg(q, e)


CASES = [
    # (code, message fragment, call(regs, env))
    (1, "Invalid number of qubits", lambda r, e: capi.createQureg(0, e)),
    (1, "Invalid number of qubits", lambda r, e: capi.createDensityQureg(-1, e)),
    (2, "Invalid target qubit", lambda r, e: capi.hadamard(r["q"], 3)),
    (2, "Invalid target qubit", lambda r, e: capi.rotateX(r["q"], -1, 0.1)),
    (2, "Invalid target qubit", lambda r, e: capi.calcProbOfOutcome(r["q"], 5, 0)),
    (3, "Invalid control qubit", lambda r, e: capi.controlledNot(r["q"], 7, 0)),
    (3, "Invalid control qubit", lambda r, e: capi.multiControlledPhaseFlip(r["q"], [0, 9], 2)),
    (4, "Invalid state index", lambda r, e: capi.getAmp(r["q"], 8)),
    (4, "Invalid state index", lambda r, e: capi.initClassicalState(r["q"], -1)),
    (4, "Invalid state index", lambda r, e: capi.getDensityAmp(r["d"], 8, 0)),
    (5, "Invalid number of amplitudes", lambda r, e: capi.setAmps(r["q"], 0, [0.0] * 9, [0.0] * 9, 9)),
    (6, "More amplitudes given", lambda r, e: capi.setAmps(r["q"], 6, [0.0] * 4, [0.0] * 4, 4)),
    (7, "Control qubit cannot equal target", lambda r, e: capi.controlledNot(r["q"], 1, 1)),
    (7, "Control qubit cannot equal target", lambda r, e: capi.controlledRotateZ(r["q"], 2, 2, 0.5)),
    (8, "Control qubits cannot include target",
     lambda r, e: capi.multiControlledUnitary(r["q"], [0, 1], 2, 1, I2)),
    (9, "target qubits must be unique", lambda r, e: capi.applyTwoQubitDephaseError(r["d"], 1, 1, 0.1)),
    (10, "Invalid number of control qubits", lambda r, e: capi.multiControlledPhaseShift(r["q"], [0], 0, 0.2)),
    (10, "Invalid number of control qubits",
     lambda r, e: capi.multiControlledPhaseFlip(r["q"], [0, 1, 2, 0], 4)),
    (11, "Matrix is not unitary", lambda r, e: capi.unitary(r["q"], 0, [[1, 1], [0, 1]])),
    (11, "Matrix is not unitary", lambda r, e: capi.controlledUnitary(r["q"], 1, 0, [[2, 0], [0, 1]])),
    (12, "Compact matrix formed by given complex numbers is not unitary",
     lambda r, e: capi.compactUnitary(r["q"], 0, 1, 1)),
    (13, "Invalid axis vector", lambda r, e: capi.rotateAroundAxis(r["q"], 0, 0.3, (0, 0, 0))),
    (15, "Can't collapse to state with zero probability", lambda r, e: capi.collapseToOutcome(r["q4"], 0, 1)),
    (16, "Invalid measurement outcome", lambda r, e: capi.calcProbOfOutcome(r["q"], 0, 2)),
    (16, "Invalid measurement outcome", lambda r, e: capi.collapseToOutcome(r["q"], 0, -1)),
    (17, "Could not open file", lambda r, e: capi.initStateFromSingleFile(r["q"], "/nonexistent/amps.csv", e)),
    (18, "Second argument must be a state-vector", lambda r, e: capi.initPureState(r["d"], r["d2"])),
    (19, "Dimensions of the qubit registers don't match", lambda r, e: capi.cloneQureg(r["q"], r["q4"])),
    (19, "Dimensions of the qubit registers don't match", lambda r, e: capi.calcInnerProduct(r["q"], r["q4"])),
    (20, "both be state-vectors or both be density", lambda r, e: capi.cloneQureg(r["q"], r["d"])),
    (21, "Operation valid only for state-vectors", lambda r, e: capi.calcInnerProduct(r["d"], r["d2"])),
    (21, "Operation valid only for state-vectors", lambda r, e: capi.getAmp(r["d"], 0)),
    (22, "Operation valid only for density matrices", lambda r, e: capi.calcPurity(r["q"])),
    (22, "Operation valid only for density matrices", lambda r, e: capi.applyOneQubitDephaseError(r["q"], 0, 0.1)),
    (22, "Operation valid only for density matrices", lambda r, e: capi.getDensityAmp(r["q"], 0, 0)),
    (23, "Probabilities must be in [0, 1]", lambda r, e: capi.applyOneQubitDampingError(r["d"], 0, -0.1)),
    (23, "Probabilities must be in [0, 1]", lambda r, e: capi.addDensityMatrix(r["d"], 1.5, r["d2"])),
    (25, "single qubit dephase error cannot exceed 1/2",
     lambda r, e: capi.applyOneQubitDephaseError(r["d"], 0, 0.6)),
    (26, "two-qubit qubit dephase error cannot exceed 3/4",
     lambda r, e: capi.applyTwoQubitDephaseError(r["d"], 0, 1, 0.8)),
    (27, "single qubit depolarising error cannot exceed 3/4",
     lambda r, e: capi.applyOneQubitDepolariseError(r["d"], 0, 0.8)),
    (28, "two-qubit depolarising error cannot exceed 15/16",
     lambda r, e: capi.applyTwoQubitDepolariseError(r["d"], 0, 1, 0.95)),
]


@pytest.mark.parametrize("code,msg,call", CASES, ids=[f"E{c}-{i}" for i, (c, _, _) in enumerate(CASES)])
def test_error_codes(regs, code, msg, call):
    r, e = regs
    capi.initPlusState(r["q"])
    before = capi.getAmps(r["q"])
    with pytest.raises(QuESTError) as ei:
        call(r, e)
    assert ei.value.code == code
    assert msg in ei.value.message
    # the rejected call left the state alone
    np.testing.assert_array_equal(capi.getAmps(r["q"]), before)


def test_report_state_too_big_prints_notice(regs, capfd):
    """The reference never raises E_SYS_TOO_BIG_TO_PRINT; its host build
    prints a notice instead (QuEST_cpu.c:1275)."""
    r, e = regs
    capi.reportStateToScreen(r["q6"], e, 0)
    out = capfd.readouterr().out
    assert "will not print output for systems of more than 5 qubits" in out
    capi.initPlusState(r["q"])
    capi.reportStateToScreen(r["q"], e, 0)
    out = capfd.readouterr().out
    assert out.startswith("Reporting state [\nreal, imag\n") and out.count("\n") == 11


def test_valid_edge_inputs_accepted(regs):
    r, e = regs
    capi.applyOneQubitDephaseError(r["d"], 0, 0.5)
    capi.applyTwoQubitDephaseError(r["d"], 0, 2, 0.75)
    capi.applyOneQubitDepolariseError(r["d"], 1, 0.75)
    capi.applyTwoQubitDepolariseError(r["d"], 1, 2, 15 / 16)
    capi.applyOneQubitDampingError(r["d"], 2, 1.0)
    capi.multiControlledPhaseFlip(r["q"], [0, 1, 2], 3)
    capi.setAmps(r["q"], 5, [0.1] * 3, [0.0] * 3, 3)
    capi.rotateAroundAxis(r["q"], 0, 0.3, (0, 0, 2.0))  # any non-zero axis (normalised)
    c = 1 / math.sqrt(2)
    capi.compactUnitary(r["q"], 1, complex(c, 0), complex(0, c))


def test_default_handler_prints_and_exits_with_code():
    """No handler installed: the reference's banner on stdout and
    exit(code) (QuEST_validation.c:82-88)."""
    code = (
        "import sys\n"
        "sys.path.insert(0, %r)\n"
        "from quest_amd.ops import capi\n"
        "b = capi.binding()\n"
        "b.exit_on_error(True)\n"
        "env = capi.createQuESTEnv()\n"
        "capi.createQureg(0, env)\n"
        "print('not reached')\n" % ROOT
    )
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, QUEST_BACKEND="cpu"))
    assert out.returncode == 1
    assert out.stdout == ("!!!\nQuEST Error in function createQureg: Invalid number of qubits. Must create >0.\n"
                          "!!!\nexiting..\n")
