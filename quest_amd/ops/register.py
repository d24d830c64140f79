"""Pythonic layer over the C API: :class:`Env` and :class:`Register`.

Every method maps to one QuEST.h call (same validation, same semantics); the
state can be exported to NumPy (host) or to a PyTorch tensor on the GPU
(device-to-device copy, no host round trip).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import capi

# gate methods the compiled fast path provides (quest_amd/ops/_gatecall)
_FAST_GATES = ("h", "x", "y", "z", "s", "t", "rx", "ry", "rz", "phase", "cnot", "cy", "cz", "crx", "cry", "crz",
               "cphase")


class Env:
    """``createQuESTEnv()`` wrapper; one per process (idempotent)."""

    def __init__(self):
        self.b = capi.binding()
        self.env = capi.createQuESTEnv()

    @property
    def rank(self) -> int:
        return self.env.rank

    @property
    def num_ranks(self) -> int:
        return self.env.numRanks

    @property
    def backend(self) -> str:
        return capi.getQuESTBackend()

    def sync(self):
        capi.syncQuESTEnv(self.env)

    def report(self):
        capi.reportQuESTEnv(self.env)

    def seed(self, seeds):
        capi.seedQuEST(list(seeds))

    def close(self):
        capi.destroyQuESTEnv(self.env)

    def qureg(self, num_qubits: int) -> "Register":
        return Register(self, num_qubits)

    def density_qureg(self, num_qubits: int) -> "Register":
        return Register(self, num_qubits, density=True)


class Register:
    """A state-vector or density matrix (``Qureg``)."""

    def __init__(self, env: Env, num_qubits: int, density: bool = False):
        self.envobj = env
        self.q = (capi.createDensityQureg if density else capi.createQureg)(num_qubits, env.env)
        self._alive = True
        self._fast = None
        g = capi.binding().gatecall()
        if g is not None:
            # the gate methods below, bound to the compiled fast path (same C
            # functions, validation and errors; src/py/gatecall.c)
            self._fast = g.bind(C.addressof(self.q), C.sizeof(self.q))
            for name in _FAST_GATES:
                setattr(self, name, getattr(self._fast, name))

    # -- properties --------------------------------------------------------
    @property
    def num_qubits(self) -> int:
        return self.q.numQubitsRepresented

    @property
    def is_density(self) -> bool:
        return bool(self.q.isDensityMatrix)

    @property
    def num_amps(self) -> int:
        return self.q.numAmpsTotal

    def close(self):
        if self._alive:
            if self._fast is not None:
                self._fast.close()
                for name in _FAST_GATES:
                    self.__dict__.pop(name, None)
                self._fast = None
            capi.destroyQureg(self.q, self.envobj.env)
            self._alive = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- init ---------------------------------------------------------------
    def init_zero(self):
        capi.initZeroState(self.q)

    def init_plus(self):
        capi.initPlusState(self.q)

    def init_classical(self, index: int):
        capi.initClassicalState(self.q, index)

    def init_pure(self, pure: "Register"):
        capi.initPureState(self.q, pure.q)

    def init_debug(self):
        capi.initStateDebug(self.q)

    def set_amps(self, amps, start: int = 0):
        a = np.asarray(amps, dtype=complex)
        if self.is_density:
            capi.setDensityAmps(self.q, a.real.ravel(order="F"), a.imag.ravel(order="F"))
        else:
            capi.setAmps(self.q, start, a.real, a.imag, len(a))

    def save(self, path):
        """Binary checkpoint (every rank writes "<path>.<rank>")."""
        return capi.saveQuregCheckpoint(self.q, path)

    def load(self, path):
        """Restore from a checkpoint written by save() on any number of ranks."""
        return capi.loadQuregCheckpoint(self.q, path)

    def clone_from(self, other: "Register"):
        capi.cloneQureg(self.q, other.q)

    # -- gates --------------------------------------------------------------
    def h(self, t):
        capi.hadamard(self.q, t)

    def x(self, t):
        capi.pauliX(self.q, t)

    def y(self, t):
        capi.pauliY(self.q, t)

    def z(self, t):
        capi.pauliZ(self.q, t)

    def s(self, t):
        capi.sGate(self.q, t)

    def t(self, t):
        capi.tGate(self.q, t)

    def rx(self, t, angle):
        capi.rotateX(self.q, t, angle)

    def ry(self, t, angle):
        capi.rotateY(self.q, t, angle)

    def rz(self, t, angle):
        capi.rotateZ(self.q, t, angle)

    def phase(self, t, angle):
        capi.phaseShift(self.q, t, angle)

    def rotate(self, t, angle, axis):
        capi.rotateAroundAxis(self.q, t, angle, axis)

    def cnot(self, c, t):
        capi.controlledNot(self.q, c, t)

    def cy(self, c, t):
        capi.controlledPauliY(self.q, c, t)

    def cz(self, a, b):
        capi.controlledPhaseFlip(self.q, a, b)

    def cphase(self, a, b, angle):
        capi.controlledPhaseShift(self.q, a, b, angle)

    def crx(self, c, t, angle):
        capi.controlledRotateX(self.q, c, t, angle)

    def cry(self, c, t, angle):
        capi.controlledRotateY(self.q, c, t, angle)

    def crz(self, c, t, angle):
        capi.controlledRotateZ(self.q, c, t, angle)

    def crotate(self, c, t, angle, axis):
        capi.controlledRotateAroundAxis(self.q, c, t, angle, axis)

    def unitary(self, t, u):
        capi.unitary(self.q, t, u)

    def compact(self, t, alpha, beta):
        capi.compactUnitary(self.q, t, alpha, beta)

    def cunitary(self, c, t, u):
        capi.controlledUnitary(self.q, c, t, u)

    def ccompact(self, c, t, alpha, beta):
        capi.controlledCompactUnitary(self.q, c, t, alpha, beta)

    def mcunitary(self, controls, t, u):
        capi.multiControlledUnitary(self.q, list(controls), len(controls), t, u)

    def mcphase(self, qubits, angle):
        capi.multiControlledPhaseShift(self.q, list(qubits), len(qubits), angle)

    def mcz(self, qubits):
        capi.multiControlledPhaseFlip(self.q, list(qubits), len(qubits))

    # -- noise --------------------------------------------------------------
    def dephase(self, t, p):
        capi.applyOneQubitDephaseError(self.q, t, p)

    def dephase2(self, a, b, p):
        capi.applyTwoQubitDephaseError(self.q, a, b, p)

    def depolarise(self, t, p):
        capi.applyOneQubitDepolariseError(self.q, t, p)

    def depolarise2(self, a, b, p):
        capi.applyTwoQubitDepolariseError(self.q, a, b, p)

    def damping(self, t, p):
        capi.applyOneQubitDampingError(self.q, t, p)

    def mix(self, other: "Register", prob: float):
        capi.addDensityMatrix(self.q, prob, other.q)

    # -- measurement & calculations -------------------------------------------
    def prob(self, t, outcome=1) -> float:
        return capi.calcProbOfOutcome(self.q, t, outcome)

    def collapse(self, t, outcome) -> float:
        return capi.collapseToOutcome(self.q, t, outcome)

    def measure(self, t) -> int:
        return capi.measure(self.q, t)

    def measure_with_stats(self, t):
        return capi.measureWithStats(self.q, t)

    def total_prob(self) -> float:
        return capi.calcTotalProb(self.q)

    def purity(self) -> float:
        return capi.calcPurity(self.q)

    def fidelity(self, pure: "Register") -> float:
        return capi.calcFidelity(self.q, pure.q)

    def inner(self, ket: "Register") -> complex:
        return capi.calcInnerProduct(self.q, ket.q)

    def amp(self, index) -> complex:
        return capi.getAmp(self.q, index)

    def density_amp(self, row, col) -> complex:
        return capi.getDensityAmp(self.q, row, col)

    # -- QASM -----------------------------------------------------------------
    def start_qasm(self):
        capi.startRecordingQASM(self.q)

    def stop_qasm(self):
        capi.stopRecordingQASM(self.q)

    @property
    def qasm(self) -> str:
        return capi.getRecordedQASM(self.q)

    # -- execution control ----------------------------------------------------
    def flush(self):
        capi.flushQureg(self.q)

    def sync(self):
        capi.syncQureg(self.q)

    # -- export ---------------------------------------------------------------
    def to_numpy(self) -> np.ndarray:
        """Full state (every rank gets all amplitudes): vector or matrix."""
        a = capi.getAmps(self.q, 0, self.q.numAmpsTotal)
        if self.is_density:
            d = 1 << self.num_qubits
            return a.reshape(d, d, order="F")  # element (r, c) at r + c*2^n
        return a

    def to_torch(self):
        """This rank's chunk as a complex PyTorch tensor on the state's device
        (device-to-device copy on the HIP build)."""
        import torch

        b = capi.binding()
        n = self.q.numAmpsPerChunk
        if b.prec == 4:
            # long double has no torch dtype: through host buffers, as complex128
            re = np.empty(n, dtype=b.np_real)
            im = np.empty(n, dtype=b.np_real)
            capi._call("copyChunkToBuffers", self.q, re.ctypes.data_as(C.c_void_p), im.ctypes.data_as(C.c_void_p))
            return torch.complex(torch.from_numpy(re.astype(np.float64)), torch.from_numpy(im.astype(np.float64)))
        dt = torch.float64 if b.prec == 2 else torch.float32
        if b.backend == "hip":
            re = torch.empty(n, dtype=dt, device="cuda")
            im = torch.empty(n, dtype=dt, device="cuda")
            capi._call("copyChunkToBuffers", self.q, C.c_void_p(re.data_ptr()), C.c_void_p(im.data_ptr()))
        else:
            re = torch.empty(n, dtype=dt)
            im = torch.empty(n, dtype=dt)
            capi._call("copyChunkToBuffers", self.q, C.c_void_p(re.data_ptr()), C.c_void_p(im.data_ptr()))
        return torch.complex(re, im)

    def from_torch(self, t):
        """Overwrite this rank's chunk from a complex tensor on the state's device."""
        import torch

        b = capi.binding()
        if b.prec == 4:
            re = np.ascontiguousarray(t.real.cpu().numpy(), dtype=b.np_real)
            im = np.ascontiguousarray(t.imag.cpu().numpy(), dtype=b.np_real)
            capi._call("copyChunkFromBuffers", self.q, re.ctypes.data_as(C.c_void_p), im.ctypes.data_as(C.c_void_p))
            return
        dt = torch.float64 if b.prec == 2 else torch.float32
        re = t.real.to(dt).contiguous()
        im = t.imag.to(dt).contiguous()
        capi._call("copyChunkFromBuffers", self.q, C.c_void_p(re.data_ptr()), C.c_void_p(im.data_ptr()))
