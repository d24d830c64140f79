"""QASM recording: the text of every recorded operation, as the reference's
recorder writes it (QuEST_qasm.c: header :70-74, gate lines :125-163 with
REAL_QASM_FORMAT "%.14g" for fp64, controlled phase / unitary global-phase
fix-ups :239-330, measurement :362-378, init :380-428; which API call records
what: QuEST.c:92-588)."""
import math
import os

import pytest

from quest_amd.ops import capi

HDR3 = "OPENQASM 2.0;\nqreg q[3];\ncreg c[3];\n"


@pytest.fixture
def q(env):
    r = capi.createQureg(3, env.env)
    capi.startRecordingQASM(r)
    yield r
    capi.destroyQureg(r, env.env)


def rec(q):
    return capi.getRecordedQASM(q)


def test_header_and_plain_gates(q):
    capi.hadamard(q, 0)
    capi.pauliX(q, 1)
    capi.pauliY(q, 2)
    capi.pauliZ(q, 0)
    capi.sGate(q, 1)
    capi.tGate(q, 2)
    assert rec(q) == HDR3 + "h q[0];\nx q[1];\ny q[2];\nz q[0];\ns q[1];\nt q[2];\n"


def test_parametrised_and_controlled(q):
    capi.rotateX(q, 2, 0.5)
    capi.rotateY(q, 0, -1.25)
    capi.rotateZ(q, 1, math.pi)
    capi.controlledNot(q, 1, 0)
    capi.controlledPauliY(q, 0, 2)
    capi.controlledPhaseFlip(q, 2, 1)
    capi.controlledRotateX(q, 0, 1, 0.125)
    capi.controlledRotateZ(q, 0, 2, 0.25)
    assert rec(q) == HDR3 + (
        "Rx(0.5) q[2];\nRy(-1.25) q[0];\nRz(3.1415926535898) q[1];\n"
        "cx q[1],q[0];\ncy q[0],q[2];\ncz q[2],q[1];\n"
        "cRx(0.125) q[0],q[1];\ncRz(0.25) q[0],q[2];\n")


def test_phase_shift_fixups(q):
    capi.phaseShift(q, 1, 0.3)
    capi.controlledPhaseShift(q, 0, 1, 0.5)
    capi.multiControlledPhaseShift(q, [2, 0, 1], 3, 0.75)
    capi.multiControlledPhaseFlip(q, [1, 2, 0], 3)
    assert rec(q) == HDR3 + (
        "Rz(0.3) q[1];\n"
        "cRz(0.5) q[0],q[1];\n"
        "// Restoring the discarded global phase of the previous controlled phase gate\n"
        "Rz(0.25) q[1];\n"
        "ccRz(0.75) q[2],q[0],q[1];\n"
        "// Restoring the discarded global phase of the previous multicontrolled phase gate\n"
        "Rz(0.375) q[1];\n"
        "ccz q[1],q[2],q[0];\n")


def test_unitaries_as_zyz(q):
    # Hadamard-like unitary: U = exp(i*pi/2) * Rz Ry Rz ...; check line shapes and
    # that the controlled unitary gets its global-phase Rz after a comment
    c = 1 / math.sqrt(2)
    capi.compactUnitary(q, 0, complex(c, 0), complex(c, 0))
    capi.unitary(q, 1, [[c, c], [c, -c]])
    capi.controlledUnitary(q, 0, 2, [[c, c], [c, -c]])
    capi.multiControlledUnitary(q, [0, 1], 2, 2, [[1, 0], [0, 1j]])
    capi.rotateAroundAxis(q, 1, 0.5, (0, 0, 1))
    capi.controlledRotateAroundAxis(q, 2, 0, 0.5, (1, 0, 0))
    lines = rec(q)[len(HDR3):].splitlines()
    assert lines[0].startswith("U(") and lines[0].endswith(") q[0];")
    assert lines[1].startswith("U(") and lines[1].endswith(") q[1];")
    assert lines[2].startswith("cU(") and lines[2].endswith(") q[0],q[2];")
    assert lines[3] == "// Restoring the discarded global phase of the previous controlled unitary"
    assert lines[4].startswith("Rz(") and lines[4].endswith(") q[2];")
    assert lines[5].startswith("ccU(") and lines[5].endswith(") q[0],q[1],q[2];")
    assert lines[6].startswith("Rz(") and lines[6].endswith(") q[2];")   # no comment for multi-controlled
    assert lines[7].startswith("U(") and lines[7].endswith(") q[1];")
    assert lines[8].startswith("cU(") and lines[8].endswith(") q[2],q[0];")
    assert len(lines) == 9
    # ZYZ angles of Rz(0.5) = exp(-i 0.25 Z): U(rz2, 0, rz1) with rz1 + rz2 = 0.5 (mod 2pi)
    params = [float(x) for x in lines[7][2:lines[7].index(")")].split(",")]
    assert params[1] == pytest.approx(0.0, abs=1e-7)  # 2*acos(|alpha|) near 1
    assert math.remainder(params[0] + params[2] - 0.5, 2 * math.pi) == pytest.approx(0.0, abs=1e-12)


def test_init_and_measurement_records(env, q):
    capi.initZeroState(q)
    capi.initPlusState(q)
    capi.initClassicalState(q, 5)
    capi.measure(q, 0)
    capi.collapseToOutcome(q, 1, 0)
    capi.measureWithStats(q, 2)
    capi.setAmps(q, 0, [1.0], [0.0], 1)
    p = capi.createQureg(3, env.env)
    capi.initPureState(q, p)
    capi.destroyQureg(p, env.env)
    assert rec(q) == HDR3 + (
        "reset q;\n"
        "// Initialising state |+>\nreset q;\nh q;\n"
        "// Initialising state |5>\nreset q;\nx q[0];\nx q[2];\n"
        "measure q[0] -> c[0];\nmeasure q[1] -> c[1];\nmeasure q[2] -> c[2];\n"
        "// Here, some amplitudes in the statevector were manually edited.\n"
        "// Here, the register was initialised to an undisclosed given pure state.\n")


def test_stop_clear_and_write(q, tmp_path):
    capi.hadamard(q, 0)
    capi.stopRecordingQASM(q)
    capi.hadamard(q, 1)  # not recorded
    assert rec(q) == HDR3 + "h q[0];\n"
    path = tmp_path / "circ.qasm"
    capi.writeRecordedQASMToFile(q, str(path))
    assert path.read_text() == HDR3 + "h q[0];\n"
    capi.clearRecordedQASM(q)  # the reference clears the header too (QuEST_qasm.c:431-435)
    assert rec(q) == ""
    capi.startRecordingQASM(q)
    capi.tGate(q, 2)
    assert rec(q) == "t q[2];\n"


def test_buffer_grows_for_long_circuits(q):
    for i in range(500):
        capi.rotateY(q, i % 3, 0.001 * i)
    text = rec(q)
    assert text.count("\n") == 3 + 500
    assert text.endswith("Ry(0.499) q[1];\n")


def test_print_recorded(q, capfd):
    capi.hadamard(q, 2)
    capi.printRecordedQASM(q)
    assert capfd.readouterr().out == HDR3 + "h q[2];\n"


def test_density_matrix_records_once(env):
    d = capi.createDensityQureg(2, env.env)
    capi.startRecordingQASM(d)
    capi.hadamard(d, 1)
    capi.controlledNot(d, 1, 0)
    assert capi.getRecordedQASM(d) == "OPENQASM 2.0;\nqreg q[2];\ncreg c[2];\nh q[1];\ncx q[1],q[0];\n"
    capi.destroyQureg(d, env.env)


def test_write_to_bad_path_raises(q):
    with pytest.raises(capi.QuESTError) as ei:
        capi.writeRecordedQASMToFile(q, os.path.join("/nonexistent", "dir", "x.qasm"))
    assert ei.value.code == 17
