"""Circuit families ("models" of this framework): a tiny gate-list IR plus
generators for the workloads the reference ships or benchmarks.

* :func:`random_layered` - depth-D random circuit: a random single-qubit gate
  on every qubit, then a CNOT brick layer (the bench.py workload);
* :func:`fork_circuit` - the zhaozzz-160 fork's exact 30-qubit benchmark
  circuit (tutorial_example.c:29-518, 490 gates; the program then takes 30
  calcProbOfOutcome and 10 getAmp), read from examples/data;
* :func:`fork_benchmark` - a seeded random circuit with the same gate-type
  histogram, for other qubit counts;
* :func:`qft`, :func:`ghz`, :func:`bernstein_vazirani` - the algorithms of the
  reference's tests/algor and examples/bernstein_vazirani_circuit.c.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np

from ..utils import oracle as O

ONE_QUBIT = ("h", "x", "y", "z", "s", "t", "rx", "ry", "rz")


@dataclass
class Gate:
    name: str
    qubits: tuple
    param: float | None = None


@dataclass
class Circuit:
    n: int
    gates: list = field(default_factory=list)

    def add(self, name, *qubits, param=None):
        self.gates.append(Gate(name, tuple(int(q) for q in qubits), param))
        return self

    def __len__(self):
        return len(self.gates)

    def count(self):
        out = {}
        for g in self.gates:
            out[g.name] = out.get(g.name, 0) + 1
        return out

    # -- execution ---------------------------------------------------------
    def apply(self, reg):
        """Apply to a quest_amd Register (one API call per gate; each gate
        name's method is looked up once per call)."""
        methods = {}
        for g in self.gates:
            name = g.name
            f = methods.get(name)
            if f is None:
                f = methods[name] = getattr(reg, name)
            if name == "mcz":
                f(list(g.qubits))
            elif g.param is None:
                f(*g.qubits)
            else:
                f(*g.qubits, g.param)

    def apply_oracle(self, o):
        """Apply to an oracle StateVector / DensityMatrix."""
        mats = {"h": O.H, "x": O.X, "y": O.Y, "z": O.Z, "s": O.S, "t": O.T}
        for g in self.gates:
            q = g.qubits
            if g.name in mats:
                o.apply(mats[g.name], q[0])
            elif g.name in ("rx", "ry", "rz"):
                axis = {"rx": (1, 0, 0), "ry": (0, 1, 0), "rz": (0, 0, 1)}[g.name]
                o.apply(O.rot(g.param, axis), q[0])
            elif g.name == "phase":
                o.apply(O.phase(g.param), q[0])
            elif g.name in ("cnot", "cy", "cz"):
                o.apply({"cnot": O.X, "cy": O.Y, "cz": O.Z}[g.name], q[1], [q[0]])
            elif g.name in ("crx", "cry", "crz"):
                axis = {"crx": (1, 0, 0), "cry": (0, 1, 0), "crz": (0, 0, 1)}[g.name]
                o.apply(O.rot(g.param, axis), q[1], [q[0]])
            elif g.name == "cphase":
                o.apply(O.phase(g.param), q[1], [q[0]])
            elif g.name == "mcz":
                o.apply(O.Z, q[-1], list(q[:-1]))
            else:
                raise ValueError(g.name)

    def inverse(self) -> "Circuit":
        """The adjoint circuit: gates reversed, each replaced by its inverse
        (so ``c`` followed by ``c.inverse()`` is the identity)."""
        inv = Circuit(self.n)
        for g in reversed(self.gates):
            if g.name in ("h", "x", "y", "z", "cnot", "cy", "cz", "mcz"):
                inv.gates.append(Gate(g.name, g.qubits))
            elif g.name == "s":
                inv.gates.append(Gate("phase", g.qubits, -math.pi / 2))
            elif g.name == "t":
                inv.gates.append(Gate("phase", g.qubits, -math.pi / 4))
            elif g.param is not None:
                inv.gates.append(Gate(g.name, g.qubits, -g.param))
            else:
                raise ValueError(f"no inverse for {g.name}")
        return inv

    def to_qasm(self) -> str:
        lines = ["OPENQASM 2.0;", f"qreg q[{self.n}];", f"creg c[{self.n}];"]
        for g in self.gates:
            args = ",".join(f"q[{q}]" for q in g.qubits)
            name = {"cnot": "cx", "phase": "u1"}.get(g.name, g.name)
            p = f"({g.param:.14g})" if g.param is not None else ""
            lines.append(f"{name}{p} {args};")
        return "\n".join(lines) + "\n"


def random_layered(n: int, depth: int, seed: int = 0, entangle: bool = True) -> Circuit:
    """Depth-`depth` random circuit: each layer applies a random single-qubit
    gate (from ONE_QUBIT, random angles) to every qubit, then CNOTs on a brick
    pattern of neighbouring pairs."""
    rng = np.random.default_rng(seed)
    c = Circuit(n)
    for layer in range(depth):
        for q in range(n):
            name = ONE_QUBIT[rng.integers(len(ONE_QUBIT))]
            if name in ("rx", "ry", "rz"):
                c.add(name, q, param=float(rng.uniform(0, 2 * math.pi)))
            else:
                c.add(name, q)
        if entangle:
            for a in range(layer % 2, n - 1, 2):
                c.add("cnot", a, a + 1)
    return c


def random_mixed(n: int, num_gates: int, seed: int = 0, high: int = 0) -> Circuit:
    """`num_gates` random gates mixing one-qubit gates, controlled gates,
    controlled rotations and multi-controlled phase flips.  With high > 0,
    targets and controls are drawn from the top `high` qubits two times in
    three (tile bits far above the low, always-resident positions)."""
    rng = np.random.default_rng(seed)
    c = Circuit(n)
    top = list(range(max(0, n - high), n)) if high > 0 else []

    def qubit():
        if top and rng.random() < 2 / 3:
            return int(top[rng.integers(len(top))])
        return int(rng.integers(n))

    def distinct(k):
        out = []
        while len(out) < k:
            q = qubit()
            if q not in out:
                out.append(q)
        return out

    kinds = ONE_QUBIT + ("phase", "cnot", "cy", "cz", "crx", "cry", "crz", "cphase", "mcz")
    for _ in range(num_gates):
        name = kinds[rng.integers(len(kinds))]
        angle = float(rng.uniform(0, 2 * math.pi))
        if name in ("rx", "ry", "rz", "phase"):
            c.add(name, qubit(), param=angle)
        elif name in ONE_QUBIT:
            c.add(name, qubit())
        elif name in ("cnot", "cy", "cz"):
            c.add(name, *distinct(2))
        elif name == "mcz":
            c.add(name, *distinct(int(rng.integers(2, 5))))
        else:
            c.add(name, *distinct(2), param=angle)
    return c


_FORK_HISTOGRAM = {  # tutorial_example.c:29-518 of the fork (counted with grep)
    "z": 44, "y": 43, "cry": 40, "cy": 40, "t": 38, "x": 37, "rx": 35, "cnot": 33,
    "rz": 32, "crz": 32, "crx": 32, "ry": 31, "h": 28, "s": 25,
}


def fork_benchmark(seed: int = 2024, n: int = 30) -> Circuit:
    """490 gates on 30 qubits with the fork benchmark's gate-type histogram,
    in a seeded random order with random qubits and angles."""
    rng = np.random.default_rng(seed)
    names = [k for k, v in _FORK_HISTOGRAM.items() for _ in range(v)]
    rng.shuffle(names)
    c = Circuit(n)
    for name in names:
        if name in ("cry", "cy", "cnot", "crz", "crx"):
            a, b = rng.permutation(n)[:2]
            if name.startswith("cr"):
                c.add(name, a, b, param=float(rng.uniform(0, 2 * math.pi)))
            else:
                c.add(name, a, b)
        elif name in ("rx", "ry", "rz"):
            c.add(name, rng.integers(n), param=float(rng.uniform(0, 2 * math.pi)))
        else:
            c.add(name, rng.integers(n))
    return c


_API_TO_GATE = {
    "hadamard": "h", "pauliX": "x", "pauliY": "y", "pauliZ": "z", "sGate": "s", "tGate": "t",
    "rotateX": "rx", "rotateY": "ry", "rotateZ": "rz", "controlledNot": "cnot", "controlledPauliY": "cy",
    "controlledRotateX": "crx", "controlledRotateY": "cry", "controlledRotateZ": "crz",
    "controlledPhaseFlip": "cz", "phaseShift": "phase", "controlledPhaseShift": "cphase",
}


def load_api_circuit(path: str, n: int) -> Circuit:
    """Read a text circuit of QuEST API calls, one per line:
    ``<function> <qubits...> [<angle>]`` (examples/data/*.txt)."""
    c = Circuit(n)
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            name, *args = line.split()
            g = _API_TO_GATE[name]
            if g in ("rx", "ry", "rz", "phase"):
                c.add(g, int(args[0]), param=float(args[1]))
            elif g in ("crx", "cry", "crz", "cphase"):
                c.add(g, int(args[0]), int(args[1]), param=float(args[2]))
            else:
                c.add(g, *[int(a) for a in args])
    return c


FORK_CIRCUIT_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                 "examples", "data", "fork_circuit_30q.txt")


def fork_circuit() -> Circuit:
    """The fork's exact 30-qubit benchmark circuit (490 gates,
    tutorial_example.c:29-518; extracted by tools/import_fork_circuit.py)."""
    return load_api_circuit(FORK_CIRCUIT_FILE, 30)


def qft(n: int) -> Circuit:
    """Quantum Fourier transform with controlled phases (no final swaps)."""
    c = Circuit(n)
    for j in reversed(range(n)):
        c.add("h", j)
        for k in reversed(range(j)):
            c.add("cphase", k, j, param=math.pi / (1 << (j - k)))
    return c


def ghz(n: int) -> Circuit:
    c = Circuit(n).add("h", 0)
    for q in range(1, n):
        c.add("cnot", q - 1, q)
    return c


def bernstein_vazirani(secret: int, n: int) -> Circuit:
    """BV circuit on n qubits: after it, the register holds |secret>."""
    c = Circuit(n)
    for q in range(n):
        c.add("h", q)
    for q in range(n):
        if (secret >> q) & 1:
            c.add("z", q)
    for q in range(n):
        c.add("h", q)
    return c
