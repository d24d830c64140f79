"""ctypes binding of the complete QuEST C API (QuEST.h, QuEST_debug.h,
quest_amd.h).

The struct layouts mirror ``include/QuEST.h`` (identical to the reference's,
``QuEST/include/QuEST.h:26-121``), so a ``Qureg`` returned by value from C is
a real ``ctypes.Structure`` whose fields (``numQubitsRepresented``,
``numAmpsTotal``, ...) read as in C.  This plays the role of the reference's
``utilities/QuESTPy`` package, with two differences: arguments are converted
from natural Python values (lists, complex numbers, numpy arrays, 2x2
nested sequences), and invalid input raises :class:`QuESTError` instead of
terminating the interpreter (the library's error handler hook).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

from .. import _lib


class QuESTError(RuntimeError):
    """Raised when the library rejects an input (reference error codes)."""

    def __init__(self, code: int, message: str, function: str):
        super().__init__(f"{function}: {message} (code {code})")
        self.code = code
        self.message = message
        self.function = function


class _Binding:
    """Types + prototypes bound to one loaded library (one precision)."""

    def __init__(self, lib: C.CDLL):
        self.lib = lib
        self.backend = lib._quest_backend
        self.prec = lib._quest_prec
        qreal = {1: C.c_float, 2: C.c_double, 4: C.c_longdouble}[self.prec]
        self.qreal = qreal
        self.np_real = {1: np.float32, 2: np.float64, 4: np.longdouble}[self.prec]

        class Complex(C.Structure):
            _fields_ = [("real", qreal), ("imag", qreal)]

        class ComplexMatrix2(C.Structure):
            _fields_ = [("r0c0", Complex), ("r0c1", Complex), ("r1c0", Complex), ("r1c1", Complex)]

        class Vector(C.Structure):
            _fields_ = [("x", qreal), ("y", qreal), ("z", qreal)]

        class ComplexArray(C.Structure):
            _fields_ = [("real", C.POINTER(qreal)), ("imag", C.POINTER(qreal))]

        class QASMLogger(C.Structure):
            _fields_ = [("buffer", C.c_char_p), ("bufferSize", C.c_int), ("bufferFill", C.c_int),
                        ("isLogging", C.c_int)]

        class Qureg(C.Structure):
            _fields_ = [
                ("isDensityMatrix", C.c_int),
                ("numQubitsRepresented", C.c_int),
                ("numQubitsInStateVec", C.c_int),
                ("numAmpsPerChunk", C.c_longlong),
                ("numAmpsTotal", C.c_longlong),
                ("chunkId", C.c_int),
                ("numChunks", C.c_int),
                ("stateVec", ComplexArray),
                ("pairStateVec", ComplexArray),
                ("deviceStateVec", ComplexArray),
                ("firstLevelReduction", C.POINTER(qreal)),
                ("secondLevelReduction", C.POINTER(qreal)),
                ("qasmLog", C.POINTER(QASMLogger)),
            ]

        class QuESTEnv(C.Structure):
            _fields_ = [("rank", C.c_int), ("numRanks", C.c_int)]

        class QuESTStats(C.Structure):
            _fields_ = [(n, C.c_longlong) for n in
                        ("opsQueued", "passes", "fusedOps", "swaps", "bytesExchanged", "reductions",
                         "verifiedFlushes", "wavePasses", "waveOps", "waveTransposes", "relabels",
                         "globalDiags", "flushes", "marginalPasses", "waveShadowChecks",
                         "waveShadowMismatches", "permutedOps", "relayouts", "restoreRounds", "swapMicros",
                         "overlappedSwaps", "overlappedPasses", "layoutAligns", "placementProbes")]

        self.Complex, self.ComplexMatrix2, self.Vector = Complex, ComplexMatrix2, Vector
        self.ComplexArray, self.QASMLogger, self.Qureg = ComplexArray, QASMLogger, Qureg
        self.QuESTEnv, self.QuESTStats = QuESTEnv, QuESTStats

        P = C.POINTER
        i, ll, r, v = C.c_int, C.c_longlong, qreal, None
        ip, rp = P(C.c_int), P(qreal)
        Q, E, Cx, M2, Vec = Qureg, QuESTEnv, Complex, ComplexMatrix2, Vector
        self.protos = {
            # registers
            "createQureg": (Q, [i, E]), "createDensityQureg": (Q, [i, E]), "destroyQureg": (v, [Q, E]),
            "cloneQureg": (v, [Q, Q]), "getNumQubits": (i, [Q]), "getNumAmps": (i, [Q]),
            "reportState": (v, [Q]), "reportStateToScreen": (v, [Q, E, i]), "reportQuregParams": (v, [Q]),
            # init
            "initZeroState": (v, [Q]), "initPlusState": (v, [Q]), "initClassicalState": (v, [Q, ll]),
            "initPureState": (v, [Q, Q]), "initStateFromAmps": (v, [Q, rp, rp]),
            "setAmps": (v, [Q, ll, rp, rp, ll]),
            # unitaries
            "phaseShift": (v, [Q, i, r]), "controlledPhaseShift": (v, [Q, i, i, r]),
            "multiControlledPhaseShift": (v, [Q, ip, i, r]), "controlledPhaseFlip": (v, [Q, i, i]),
            "multiControlledPhaseFlip": (v, [Q, ip, i]), "sGate": (v, [Q, i]), "tGate": (v, [Q, i]),
            "compactUnitary": (v, [Q, i, Cx, Cx]), "unitary": (v, [Q, i, M2]),
            "rotateX": (v, [Q, i, r]), "rotateY": (v, [Q, i, r]), "rotateZ": (v, [Q, i, r]),
            "rotateAroundAxis": (v, [Q, i, r, Vec]),
            "controlledRotateX": (v, [Q, i, i, r]), "controlledRotateY": (v, [Q, i, i, r]),
            "controlledRotateZ": (v, [Q, i, i, r]), "controlledRotateAroundAxis": (v, [Q, i, i, r, Vec]),
            "controlledCompactUnitary": (v, [Q, i, i, Cx, Cx]), "controlledUnitary": (v, [Q, i, i, M2]),
            "multiControlledUnitary": (v, [Q, ip, i, i, M2]),
            "pauliX": (v, [Q, i]), "pauliY": (v, [Q, i]), "pauliZ": (v, [Q, i]), "hadamard": (v, [Q, i]),
            "controlledNot": (v, [Q, i, i]), "controlledPauliY": (v, [Q, i, i]),
            # env
            "createQuESTEnv": (E, []), "destroyQuESTEnv": (v, [E]), "syncQuESTEnv": (v, [E]),
            "syncQuESTSuccess": (i, [i]), "reportQuESTEnv": (v, [E]),
            "getEnvironmentString": (v, [E, Q, C.c_char_p]),
            # amplitudes / calculations
            "getAmp": (Cx, [Q, ll]), "getRealAmp": (r, [Q, ll]), "getImagAmp": (r, [Q, ll]),
            "getProbAmp": (r, [Q, ll]), "getDensityAmp": (Cx, [Q, ll, ll]), "calcTotalProb": (r, [Q]),
            "calcProbOfOutcome": (r, [Q, i, i]), "collapseToOutcome": (r, [Q, i, i]),
            "measure": (i, [Q, i]), "measureWithStats": (i, [Q, i, rp]),
            "calcInnerProduct": (Cx, [Q, Q]), "calcPurity": (r, [Q]), "calcFidelity": (r, [Q, Q]),
            # rng
            "seedQuESTDefault": (v, []), "seedQuEST": (v, [P(C.c_ulong), i]),
            "genrand_real1": (C.c_double, []), "genrand_int32": (C.c_ulong, []),
            "init_by_array": (v, [P(C.c_ulong), i]), "init_genrand": (v, [C.c_ulong]),
            # qasm
            "startRecordingQASM": (v, [Q]), "stopRecordingQASM": (v, [Q]), "clearRecordedQASM": (v, [Q]),
            "printRecordedQASM": (v, [Q]), "writeRecordedQASMToFile": (v, [Q, C.c_char_p]),
            # decoherence
            "applyOneQubitDephaseError": (v, [Q, i, r]), "applyTwoQubitDephaseError": (v, [Q, i, i, r]),
            "applyOneQubitDepolariseError": (v, [Q, i, r]), "applyOneQubitDampingError": (v, [Q, i, r]),
            "applyTwoQubitDepolariseError": (v, [Q, i, i, r]), "addDensityMatrix": (v, [Q, r, Q]),
            # debug
            "initStateOfSingleQubit": (v, [P(Q), i, i]), "initStateDebug": (v, [Q]),
            "initStateFromSingleFile": (v, [P(Q), C.c_char_p, E]), "compareStates": (i, [Q, Q, r]),
            "setDensityAmps": (v, [Q, rp, rp]), "getQuEST_PREC": (i, []),
            # MI355X extensions
            "setGateFusion": (v, [i]), "getGateFusion": (i, []), "setFusionMaxQubits": (v, [i]),
            "setQuESTTuning": (i, [C.c_char_p, i]), "getQuESTTuning": (i, [C.c_char_p, ip]),
            "getQuregMemoryPlan": (v, [i, i, P(ll)]), "runCommSelfTest": (i, [C.c_char_p, i]),
            "runFootprintCheck": (i, [i, i, C.c_char_p, i]),
            "flushQureg": (v, [Q]), "syncQureg": (v, [Q]), "copyStateToGPU": (v, [Q]),
            "copyStateFromGPU": (v, [Q]), "copyChunkToBuffers": (v, [Q, C.c_void_p, C.c_void_p]),
            "copyChunkFromBuffers": (v, [Q, C.c_void_p, C.c_void_p]), "canonicaliseQureg": (v, [Q]),
            "getQubitLayout": (v, [Q, ip]), "getAmps": (v, [Q, ll, rp, rp, ll]), "getQuESTStats": (v, [P(QuESTStats)]), "resetQuESTStats": (v, []),
            "getQuESTBackend": (C.c_char_p, []), "getQuESTTransport": (C.c_char_p, []), "getQuESTSeeds": (v, [P(C.c_ulong), ip]),
            "saveQuregCheckpoint": (i, [Q, C.c_char_p]), "loadQuregCheckpoint": (i, [Q, C.c_char_p]),
        }
        for name, (res, args) in self.protos.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args

        # every wrapped function, resolved once (the per-gate call path)
        self.fns = {name: getattr(lib, name) for name in self.protos}
        # error handler: record (per thread), then the wrapper raises; the
        # wrappers test the plain counter `nerr` (cheap) before looking
        self._err = threading.local()
        self.nerr = 0
        # the same count where the per-gate fast path (_gatecall) reads it
        self._errflag = C.c_int(0)
        self._gatecall = None
        HANDLER = C.CFUNCTYPE(None, C.c_int, C.c_char_p, C.c_char_p)

        def _handler(code, msg, func):
            self._err.value = (int(code), msg.decode(), func.decode())
            self.nerr += 1
            self._errflag.value = self.nerr

        self._handler = HANDLER(_handler)  # keep alive
        self._null_handler = HANDLER()
        lib.setQuESTErrorHandler.argtypes = [HANDLER]
        lib.setQuESTErrorHandler.restype = None
        lib.setQuESTErrorHandler(self._handler)

    def exit_on_error(self, enabled: bool = True):
        """True: the reference's behaviour (print, then exit(code));
        False (default): raise QuESTError."""
        self.lib.setQuESTErrorHandler(self._null_handler if enabled else self._handler)

    # -- conversions ---------------------------------------------------------
    def to_complex(self, z) -> "C.Structure":
        if isinstance(z, self.Complex):
            return z
        z = complex(z)
        return self.Complex(z.real, z.imag)

    def to_matrix2(self, m) -> "C.Structure":
        if isinstance(m, self.ComplexMatrix2):
            return m
        a = np.asarray(m, dtype=complex).reshape(2, 2)
        cx = self.to_complex
        return self.ComplexMatrix2(cx(a[0, 0]), cx(a[0, 1]), cx(a[1, 0]), cx(a[1, 1]))

    def to_vector(self, v) -> "C.Structure":
        if isinstance(v, self.Vector):
            return v
        x, y, z = v
        return self.Vector(x, y, z)

    def int_array(self, xs):
        xs = [int(x) for x in xs]
        return (C.c_int * len(xs))(*xs)

    def real_array(self, xs):
        a = np.ascontiguousarray(np.asarray(xs, dtype=self.np_real))
        return a, a.ctypes.data_as(C.POINTER(self.qreal))

    def check(self):
        if not self.nerr:
            return
        e = getattr(self._err, "value", None)
        if e is not None:
            self._err.value = None
            self.nerr -= 1
            self._errflag.value = self.nerr
            raise QuESTError(*e)

    def gatecall(self):
        """The compiled per-gate fast path (src/py/gatecall.c) configured for
        this library, or None (not built, or QUEST_PY_GATECALL=0): one- and
        two-qubit gate methods of a Register call the C API without ctypes."""
        if self._gatecall is None:
            self._gatecall = False
            if os.environ.get("QUEST_PY_GATECALL", "1") != "0":
                try:
                    from . import _gatecall as g
                except ImportError:
                    g = None
                if g is not None and g.qureg_size() == C.sizeof(self.Qureg):
                    addrs = [C.cast(self.fns[name], C.c_void_p).value for name in g.FUNCTIONS]
                    g.configure(addrs, self.prec, C.addressof(self._errflag), self.check)
                    self._gatecall = g
        return self._gatecall or None


_binding: _Binding | None = None


def binding(backend: str | None = None, prec: int | None = None) -> _Binding:
    """The process-wide binding (created on first use)."""
    global _binding
    if _binding is None:
        _binding = _Binding(_lib.load(backend, prec))
    return _binding


def reset_binding():
    global _binding
    _binding = None


def _call(name: str, *args):
    b = _binding if _binding is not None else binding()
    res = b.fns[name](*args) if name in b.fns else getattr(b.lib, name)(*args)
    if b.nerr:
        b.check()
    return res


def _mk(name, conv):
    def f(*args):
        return conv(binding(), *args)

    f.__name__ = name
    return f


# ---------------------------------------------------------------------------
# raw API with argument conversion (same names as the C functions)
# ---------------------------------------------------------------------------

def _cx_out(c):
    return complex(c.real, c.imag)


def _gen_wrappers():
    g = {}
    simple = [
        "createQureg", "createDensityQureg", "destroyQureg", "cloneQureg", "getNumQubits", "getNumAmps",
        "reportState", "reportStateToScreen", "reportQuregParams", "initZeroState", "initPlusState",
        "initClassicalState", "initPureState", "phaseShift", "controlledPhaseShift", "controlledPhaseFlip",
        "sGate", "tGate", "rotateX", "rotateY", "rotateZ", "controlledRotateX", "controlledRotateY",
        "controlledRotateZ", "pauliX", "pauliY", "pauliZ", "hadamard", "controlledNot", "controlledPauliY",
        "createQuESTEnv", "destroyQuESTEnv", "syncQuESTEnv", "syncQuESTSuccess", "reportQuESTEnv",
        "getRealAmp", "getImagAmp", "getProbAmp", "calcTotalProb", "calcProbOfOutcome", "collapseToOutcome",
        "measure", "calcPurity", "calcFidelity", "seedQuESTDefault", "startRecordingQASM", "stopRecordingQASM",
        "clearRecordedQASM", "printRecordedQASM", "applyOneQubitDephaseError", "applyTwoQubitDephaseError",
        "applyOneQubitDepolariseError", "applyOneQubitDampingError", "applyTwoQubitDepolariseError",
        "addDensityMatrix", "initStateDebug", "compareStates", "getQuEST_PREC", "genrand_real1", "genrand_int32",
        "init_genrand", "setGateFusion", "getGateFusion", "setFusionMaxQubits", "flushQureg", "syncQureg",
        "copyStateToGPU", "copyStateFromGPU", "canonicaliseQureg", "resetQuESTStats",
    ]
    def wrap(name):
        # the per-gate path: no conversions, one dict lookup, the counter test
        def w(*a):
            b = _binding if _binding is not None else binding()
            res = b.fns[name](*a)
            if b.nerr:
                b.check()
            return res

        w.__name__ = name
        return w

    for n in simple:
        g[n] = wrap(n)
    return g


globals().update(_gen_wrappers())


def getAmp(q, index):
    return _cx_out(_call("getAmp", q, index))


def getDensityAmp(q, row, col):
    return _cx_out(_call("getDensityAmp", q, row, col))


def calcInnerProduct(bra, ket):
    return _cx_out(_call("calcInnerProduct", bra, ket))


def compactUnitary(q, target, alpha, beta):
    b = binding()
    _call("compactUnitary", q, target, b.to_complex(alpha), b.to_complex(beta))


def controlledCompactUnitary(q, control, target, alpha, beta):
    b = binding()
    _call("controlledCompactUnitary", q, control, target, b.to_complex(alpha), b.to_complex(beta))


def unitary(q, target, u):
    _call("unitary", q, target, binding().to_matrix2(u))


def controlledUnitary(q, control, target, u):
    _call("controlledUnitary", q, control, target, binding().to_matrix2(u))


def multiControlledUnitary(q, controls, numControls, target, u=None):
    # accepts (q, controls, target, u) too
    if u is None:
        numControls, target, u = len(controls), numControls, target
    b = binding()
    _call("multiControlledUnitary", q, b.int_array(controls), numControls, target, b.to_matrix2(u))


def multiControlledPhaseShift(q, controls, numControls, angle=None):
    if angle is None:
        numControls, angle = len(controls), numControls
    _call("multiControlledPhaseShift", q, binding().int_array(controls), numControls, angle)


def multiControlledPhaseFlip(q, controls, numControls=None):
    if numControls is None:
        numControls = len(controls)
    _call("multiControlledPhaseFlip", q, binding().int_array(controls), numControls)


def rotateAroundAxis(q, target, angle, axis):
    _call("rotateAroundAxis", q, target, angle, binding().to_vector(axis))


def controlledRotateAroundAxis(q, control, target, angle, axis):
    _call("controlledRotateAroundAxis", q, control, target, angle, binding().to_vector(axis))


def initStateFromAmps(q, reals, imags):
    b = binding()
    ra, rp = b.real_array(reals)
    ia, ipt = b.real_array(imags)
    _call("initStateFromAmps", q, rp, ipt)


def setAmps(q, startInd, reals, imags, numAmps=None):
    b = binding()
    ra, rp = b.real_array(reals)
    ia, ipt = b.real_array(imags)
    if numAmps is None:
        numAmps = len(ra)
    _call("setAmps", q, startInd, rp, ipt, numAmps)


def setDensityAmps(q, reals, imags):
    b = binding()
    ra, rp = b.real_array(reals)
    ia, ipt = b.real_array(imags)
    _call("setDensityAmps", q, rp, ipt)


def measureWithStats(q, target):
    """Returns (outcome, probability)."""
    b = binding()
    p = b.qreal(0)
    out = _call("measureWithStats", q, target, C.byref(p))
    return out, float(p.value)


def seedQuEST(seeds, numSeeds=None):
    seeds = [int(s) for s in seeds]
    n = len(seeds) if numSeeds is None else numSeeds
    _call("seedQuEST", (C.c_ulong * len(seeds))(*seeds), n)


def init_by_array(seeds):
    seeds = [int(s) for s in seeds]
    _call("init_by_array", (C.c_ulong * len(seeds))(*seeds), len(seeds))


def getEnvironmentString(env, q) -> str:
    buf = C.create_string_buffer(200)
    _call("getEnvironmentString", env, q, buf)
    return buf.value.decode()


def writeRecordedQASMToFile(q, filename):
    _call("writeRecordedQASMToFile", q, str(filename).encode())


def getRecordedQASM(q) -> str:
    """The QASM buffer of a register as a Python string."""
    log = q.qasmLog.contents
    return (log.buffer or b"").decode()


def initStateOfSingleQubit(q, qubit, outcome):
    _call("initStateOfSingleQubit", C.byref(q), qubit, outcome)


def initStateFromSingleFile(q, filename, env):
    _call("initStateFromSingleFile", C.byref(q), str(filename).encode(), env)


def getAmps(q, startInd=0, numAmps=None):
    """Amplitudes [startInd, startInd+numAmps) as a complex numpy array."""
    b = binding()
    if numAmps is None:
        numAmps = q.numAmpsTotal - startInd
    re = np.empty(numAmps, dtype=b.np_real)
    im = np.empty(numAmps, dtype=b.np_real)
    _call("getAmps", q, startInd, re.ctypes.data_as(C.POINTER(b.qreal)), im.ctypes.data_as(C.POINTER(b.qreal)),
          numAmps)
    return re.astype(np.float64) + 1j * im.astype(np.float64)


def getQuESTStats() -> dict:
    b = binding()
    s = b.QuESTStats()
    _call("getQuESTStats", C.byref(s))
    return {n: getattr(s, n) for n, _ in b.QuESTStats._fields_}


def setQuESTTuning(key: str, value: int) -> bool:
    return bool(_call("setQuESTTuning", key.encode(), int(value)))


def getQuregMemoryPlan(num_qubits_in_statevec: int, num_ranks: int = 0) -> dict:
    """Per-rank device bytes of a register on num_ranks ranks (0: this job's):
    state, exchange, scratch, total."""
    out = (C.c_longlong * 4)()
    _call("getQuregMemoryPlan", int(num_qubits_in_statevec), int(num_ranks), out)
    return dict(zip(("state", "exchange", "scratch", "total"), list(out)))


def runCommSelfTest():
    """(ok, report) of the device transport self-test (quest_amd.h)."""
    buf = C.create_string_buffer(512)
    ok = _call("runCommSelfTest", buf, 512)
    return bool(ok), buf.value.decode()


def runFootprintCheck(num_qubits_in_statevec: int, num_ranks: int):
    """(ok, report) of the per-rank footprint check (quest_amd.h)."""
    buf = C.create_string_buffer(1024)
    ok = _call("runFootprintCheck", int(num_qubits_in_statevec), int(num_ranks), buf, 1024)
    return bool(ok), buf.value.decode()


def getQuESTTuning(key: str):
    """Current value of a tuning knob, or None if the build does not know it."""
    v = C.c_int(0)
    return v.value if _call("getQuESTTuning", key.encode(), C.byref(v)) else None


def getQuESTBackend() -> str:
    return _call("getQuESTBackend").decode()


def getQuESTTransport() -> str:
    return _call("getQuESTTransport").decode()


def saveQuregCheckpoint(q, path) -> bool:
    return bool(_call("saveQuregCheckpoint", q, str(path).encode()))


def loadQuregCheckpoint(q, path) -> bool:
    return bool(_call("loadQuregCheckpoint", q, str(path).encode()))


def getQubitLayout(q) -> list:
    n = q.numQubitsInStateVec
    arr = (C.c_int * n)()
    _call("getQubitLayout", q, arr)
    return list(arr)


def getQuESTSeeds() -> list:
    seeds = (C.c_ulong * 64)()
    n = C.c_int(0)
    _call("getQuESTSeeds", seeds, C.byref(n))
    return list(seeds[: n.value])
