"""Independent NumPy reference simulator used as the test oracle.

Unlike the reference's golden files (which the reference generated with its
own library), this oracle is written from the physics: gates
are explicit matrices applied by tensor contraction, density matrices evolve
as U rho U^dag and noise channels through their Kraus operators.  Qubit q is
bit q of the amplitude index; rho[r, c] is stored at flat index r + c 2^n.
"""
from __future__ import annotations

import math

import numpy as np

I2 = np.eye(2, dtype=complex)
X = np.array([[0, 1], [1, 0]], dtype=complex)
Y = np.array([[0, -1j], [1j, 0]], dtype=complex)
Z = np.array([[1, 0], [0, -1]], dtype=complex)
H = np.array([[1, 1], [1, -1]], dtype=complex) / math.sqrt(2)
S = np.diag([1, 1j])
T = np.diag([1, np.exp(1j * math.pi / 4)])


def rot(angle, axis):
    n = np.asarray(axis, dtype=float)
    n = n / np.linalg.norm(n)
    return math.cos(angle / 2) * I2 - 1j * math.sin(angle / 2) * (n[0] * X + n[1] * Y + n[2] * Z)


def compact(alpha, beta):
    return np.array([[alpha, -np.conj(beta)], [beta, np.conj(alpha)]], dtype=complex)


def phase(angle):
    return np.diag([1, np.exp(1j * angle)])


def random_unitary(rng, dim=2):
    z = (rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))) / math.sqrt(2)
    q, r = np.linalg.qr(z)
    d = np.diag(r)
    return q * (d / abs(d))


def random_state(rng, n):
    v = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    return v / np.linalg.norm(v)


def random_density(rng, n, rank=3):
    rho = np.zeros((1 << n, 1 << n), dtype=complex)
    w = rng.random(rank)
    w /= w.sum()
    for k in range(rank):
        v = random_state(rng, n)
        rho += w[k] * np.outer(v, v.conj())
    return rho


def full_operator(n, targets, m, controls=()):
    """Dense 2^n x 2^n matrix of m acting on `targets` (targets[0] = lowest
    bit of m's index), controlled on `controls` (all must be 1)."""
    dim = 1 << n
    k = len(targets)
    out = np.zeros((dim, dim), dtype=complex)
    cmask = 0
    for c in controls:
        cmask |= 1 << c
    for col in range(dim):
        if (col & cmask) != cmask:
            out[col, col] = 1
            continue
        sub = 0
        for j, t in enumerate(targets):
            sub |= ((col >> t) & 1) << j
        base = col
        for t in targets:
            base &= ~(1 << t)
        for row_sub in range(1 << k):
            row = base
            for j, t in enumerate(targets):
                row |= ((row_sub >> j) & 1) << t
            out[row, col] += m[row_sub, sub]
    return out


class StateVector:
    def __init__(self, n, amps=None):
        self.n = n
        self.v = np.zeros(1 << n, dtype=complex) if amps is None else np.array(amps, dtype=complex)
        if amps is None:
            self.v[0] = 1

    def apply(self, m, targets, controls=()):
        targets = [targets] if np.isscalar(targets) else list(targets)
        self.v = _apply_vec(self.v, self.n, np.asarray(m, dtype=complex), targets, list(controls))

    def prob(self, q, outcome):
        idx = np.arange(1 << self.n)
        sel = ((idx >> q) & 1) == outcome
        return float(np.sum(np.abs(self.v[sel]) ** 2))

    def collapse(self, q, outcome):
        idx = np.arange(1 << self.n)
        p = self.prob(q, outcome)
        self.v = np.where(((idx >> q) & 1) == outcome, self.v / math.sqrt(p), 0)
        return p


def _apply_vec(v, n, m, targets, controls):
    """Apply m on `targets` with `controls` to the vector v (tensor form)."""
    psi = v.reshape([2] * n)  # axis a <-> qubit n-1-a
    k = len(targets)
    ax_t = [n - 1 - t for t in targets]
    # build index of controlled subspace
    sl = [slice(None)] * n
    for c in controls:
        sl[n - 1 - c] = 1
    sub = psi[tuple(sl)].copy() if controls else psi.copy()
    # remaining axes after fixing controls
    remaining = [a for a in range(n) if a not in [n - 1 - c for c in controls]]
    ax_sub = [remaining.index(a) for a in ax_t]
    # move target axes to front in order targets[k-1], ..., targets[0] (m index bits)
    order = list(reversed(ax_sub))
    sub_m = np.moveaxis(sub, order, list(range(k)))
    shp = sub_m.shape
    flat = sub_m.reshape(1 << k, -1)
    flat = m @ flat
    sub_m = flat.reshape(shp)
    sub = np.moveaxis(sub_m, list(range(k)), order)
    if controls:
        psi = psi.copy()
        psi[tuple(sl)] = sub
    else:
        psi = sub
    return psi.reshape(-1)


class DensityMatrix:
    """rho as a (2^n, 2^n) matrix; flat() gives the QuEST column-major layout."""

    def __init__(self, n, rho=None):
        self.n = n
        if rho is None:
            self.rho = np.zeros((1 << n, 1 << n), dtype=complex)
            self.rho[0, 0] = 1
        else:
            self.rho = np.array(rho, dtype=complex)

    def flat(self):
        return self.rho.reshape(-1, order="F")

    def apply(self, m, targets, controls=()):
        targets = [targets] if np.isscalar(targets) else list(targets)
        U = full_operator(self.n, targets, np.asarray(m, dtype=complex), controls)
        self.rho = U @ self.rho @ U.conj().T

    def kraus(self, ops, targets):
        targets = [targets] if np.isscalar(targets) else list(targets)
        new = np.zeros_like(self.rho)
        for K in ops:
            U = full_operator(self.n, targets, K)
            new += U @ self.rho @ U.conj().T
        self.rho = new

    def dephase(self, q, p):
        self.kraus([math.sqrt(1 - p) * I2, math.sqrt(p) * Z], q)

    def depolarise(self, q, p):
        self.kraus([math.sqrt(1 - p) * I2] + [math.sqrt(p / 3) * P for P in (X, Y, Z)], q)

    def damping(self, q, p):
        self.kraus([np.array([[1, 0], [0, math.sqrt(1 - p)]]), np.array([[0, math.sqrt(p)], [0, 0]])], q)

    def dephase2(self, a, b, p):
        ZZ = np.kron(Z, Z)
        ops = [math.sqrt(1 - p) * np.eye(4)] + [math.sqrt(p / 3) * K for K in (np.kron(I2, Z), np.kron(Z, I2), ZZ)]
        # np.kron(A, B) acts with B on the low bit (targets[0] = a)
        self.kraus(ops, [a, b])

    def depolarise2(self, a, b, p):
        paulis = [I2, X, Y, Z]
        ops = [math.sqrt(1 - p) * np.eye(4)]
        for i, A in enumerate(paulis):
            for j, B in enumerate(paulis):
                if i == 0 and j == 0:
                    continue
                ops.append(math.sqrt(p / 15) * np.kron(A, B))
        self.kraus(ops, [a, b])

    def prob(self, q, outcome):
        idx = np.arange(1 << self.n)
        sel = ((idx >> q) & 1) == outcome
        return float(np.real(np.sum(np.diag(self.rho)[sel])))

    def collapse(self, q, outcome):
        p = self.prob(q, outcome)
        P = full_operator(self.n, [q], np.diag([1 - outcome, outcome]).astype(complex))
        self.rho = P @ self.rho @ P / p
        return p

    def purity(self):
        return float(np.real(np.trace(self.rho @ self.rho)))
