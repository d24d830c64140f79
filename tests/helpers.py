"""Shared test machinery: random op streams applied both to a quest_amd
register and to the NumPy oracle."""
from __future__ import annotations

import math

import numpy as np

from quest_amd.ops import capi
from quest_amd.utils import oracle as O


def load_state(reg, amps):
    """Write an oracle state (vector or matrix) into a register."""
    a = np.asarray(amps, dtype=complex)
    if reg.is_density:
        flat = a.reshape(-1, order="F")
        capi.setDensityAmps(reg.q, flat.real, flat.imag)
    else:
        capi.setAmps(reg.q, 0, a.real, a.imag, len(a))


def state_of(reg):
    return reg.to_numpy()


def oracle_for(reg, rng):
    n = reg.num_qubits
    if reg.is_density:
        o = O.DensityMatrix(n, O.random_density(rng, n))
    else:
        o = O.StateVector(n, O.random_state(rng, n))
    load_state(reg, o.rho if reg.is_density else o.v)
    return o


GATES_1Q = ["h", "x", "y", "z", "s", "t", "rx", "ry", "rz", "phase", "rotate", "unitary", "compact"]
GATES_2Q = ["cnot", "cy", "cz", "cphase", "crx", "cry", "crz", "crotate", "cunitary", "ccompact"]
GATES_MQ = ["mcunitary", "mcphase", "mcz"]


def apply_named(reg, o, name, qubits, rng):
    """Apply gate `name` to reg and oracle o; qubits = [ctrl..., target]."""
    angle = float(rng.uniform(-math.pi, math.pi))
    axis = tuple(rng.normal(size=3))
    U = O.random_unitary(rng)
    alpha, beta = U[0, 0], U[1, 0]
    if abs(U[0, 1] + np.conj(beta)) > 1e-9:  # ensure compact form [[a, -b*], [b, a*]]
        ph = np.exp(-1j * np.angle(np.linalg.det(U)) / 2)
        U = U * ph
        alpha, beta = U[0, 0], U[1, 0]
    t = qubits[-1]
    c = qubits[:-1]
    if name == "h":
        reg.h(t); o.apply(O.H, t)
    elif name == "x":
        reg.x(t); o.apply(O.X, t)
    elif name == "y":
        reg.y(t); o.apply(O.Y, t)
    elif name == "z":
        reg.z(t); o.apply(O.Z, t)
    elif name == "s":
        reg.s(t); o.apply(O.S, t)
    elif name == "t":
        reg.t(t); o.apply(O.T, t)
    elif name == "rx":
        reg.rx(t, angle); o.apply(O.rot(angle, (1, 0, 0)), t)
    elif name == "ry":
        reg.ry(t, angle); o.apply(O.rot(angle, (0, 1, 0)), t)
    elif name == "rz":
        reg.rz(t, angle); o.apply(O.rot(angle, (0, 0, 1)), t)
    elif name == "phase":
        reg.phase(t, angle); o.apply(O.phase(angle), t)
    elif name == "rotate":
        reg.rotate(t, angle, axis); o.apply(O.rot(angle, axis), t)
    elif name == "unitary":
        reg.unitary(t, U); o.apply(U, t)
    elif name == "compact":
        reg.compact(t, alpha, beta); o.apply(O.compact(alpha, beta), t)
    elif name == "cnot":
        reg.cnot(c[0], t); o.apply(O.X, t, c)
    elif name == "cy":
        reg.cy(c[0], t); o.apply(O.Y, t, c)
    elif name == "cz":
        reg.cz(c[0], t); o.apply(O.Z, t, c)
    elif name == "cphase":
        reg.cphase(c[0], t, angle); o.apply(O.phase(angle), t, c)
    elif name == "crx":
        reg.crx(c[0], t, angle); o.apply(O.rot(angle, (1, 0, 0)), t, c)
    elif name == "cry":
        reg.cry(c[0], t, angle); o.apply(O.rot(angle, (0, 1, 0)), t, c)
    elif name == "crz":
        reg.crz(c[0], t, angle); o.apply(O.rot(angle, (0, 0, 1)), t, c)
    elif name == "crotate":
        reg.crotate(c[0], t, angle, axis); o.apply(O.rot(angle, axis), t, c)
    elif name == "cunitary":
        reg.cunitary(c[0], t, U); o.apply(U, t, c)
    elif name == "ccompact":
        reg.ccompact(c[0], t, alpha, beta); o.apply(O.compact(alpha, beta), t, c)
    elif name == "mcunitary":
        reg.mcunitary(c, t, U); o.apply(U, t, c)
    elif name == "mcphase":
        reg.mcphase(qubits, angle); o.apply(O.phase(angle), t, c)
    elif name == "mcz":
        reg.mcz(qubits); o.apply(O.Z, t, c)
    else:
        raise ValueError(name)


def random_qubits(rng, n, k):
    return [int(x) for x in rng.permutation(n)[:k]]


def apply_random_ops(reg, o, rng, count, noise=False):
    n = reg.num_qubits
    names = GATES_1Q + GATES_2Q + GATES_MQ
    for _ in range(count):
        name = names[rng.integers(len(names))]
        if name in GATES_1Q:
            qs = random_qubits(rng, n, 1)
        elif name in GATES_2Q:
            qs = random_qubits(rng, n, 2)
        else:
            qs = random_qubits(rng, n, int(rng.integers(2, min(n, 4) + 1)))
        apply_named(reg, o, name, qs, rng)
        if noise and reg.is_density and rng.random() < 0.3:
            apply_random_noise(reg, o, rng)


def apply_random_noise(reg, o, rng):
    n = reg.num_qubits
    kind = int(rng.integers(5))
    a, b = random_qubits(rng, n, 2) if n > 1 else (0, 0)
    if kind == 0:
        p = float(rng.uniform(0, 0.5)); reg.dephase(a, p); o.dephase(a, p)
    elif kind == 1:
        p = float(rng.uniform(0, 0.75)); reg.depolarise(a, p); o.depolarise(a, p)
    elif kind == 2:
        p = float(rng.uniform(0, 1)); reg.damping(a, p); o.damping(a, p)
    elif kind == 3 and n > 1:
        p = float(rng.uniform(0, 0.75)); reg.dephase2(a, b, p); o.dephase2(a, b, p)
    elif kind == 4 and n > 1:
        p = float(rng.uniform(0, 15 / 16)); reg.depolarise2(a, b, p); o.depolarise2(a, b, p)


def assert_close(reg, o, tol=1e-10):
    got = state_of(reg)
    want = o.rho if reg.is_density else o.v
    err = np.max(np.abs(got - want))
    assert err < tol, f"max abs error {err}"
