"""Every unitary of the API against the NumPy oracle, on state-vectors and
density matrices, for every target and control placement (the reference's
tests/unit/*/gates/*.test cover 3 qubits; here 3-6 qubits, random states)."""
import itertools

import numpy as np
import pytest

import quest_amd as qa
from helpers import GATES_1Q, GATES_2Q, apply_named, apply_random_ops, assert_close, oracle_for


@pytest.mark.parametrize("name", GATES_1Q)
@pytest.mark.parametrize("density", [False, True])
def test_single_qubit_gates_every_target(env, rng, name, density):
    n = 3 if density else 5
    reg = qa.Register(env, n, density=density)
    for t in range(n):
        o = oracle_for(reg, rng)
        apply_named(reg, o, name, [t], rng)
        assert_close(reg, o)
    reg.close()


@pytest.mark.parametrize("name", GATES_2Q)
@pytest.mark.parametrize("density", [False, True])
def test_controlled_gates_every_pair(env, rng, name, density):
    n = 3 if density else 4
    reg = qa.Register(env, n, density=density)
    for c, t in itertools.permutations(range(n), 2):
        o = oracle_for(reg, rng)
        apply_named(reg, o, name, [c, t], rng)
        assert_close(reg, o)
    reg.close()


@pytest.mark.parametrize("name", ["mcunitary", "mcphase", "mcz"])
@pytest.mark.parametrize("density", [False, True])
def test_multi_controlled(env, rng, name, density):
    n = 3 if density else 5
    reg = qa.Register(env, n, density=density)
    for k in range(2, n + 1):
        for _ in range(4):
            qs = [int(x) for x in rng.permutation(n)[:k]]
            o = oracle_for(reg, rng)
            apply_named(reg, o, name, qs, rng)
            assert_close(reg, o)
    reg.close()


@pytest.mark.parametrize("density", [False, True])
def test_random_circuits(env, rng, density):
    n = 4 if density else 7
    reg = qa.Register(env, n, density=density)
    for trial in range(3):
        o = oracle_for(reg, rng)
        apply_random_ops(reg, o, rng, 60, noise=density)
        assert_close(reg, o, tol=1e-9)
    reg.close()


def test_tutorial_circuit_reference_output(env):
    """examples/README.md:146-156 of the reference."""
    r = qa.Register(env, 3)
    r.h(0)
    r.cnot(0, 1)
    r.ry(2, 0.1)
    r.mcz([0, 1, 2])
    u = [[0.5 + 0.5j, 0.5 - 0.5j], [0.5 - 0.5j, 0.5 + 0.5j]]
    r.unitary(0, u)
    r.compact(1, 0.5 + 0.5j, 0.5 - 0.5j)
    r.rotate(2, 3.14 / 2, (1, 0, 0))
    r.ccompact(0, 1, 0.5 + 0.5j, 0.5 - 0.5j)
    r.mcunitary([0, 1], 2, u)
    amp = r.amp(7)
    assert abs(abs(amp) ** 2 - 0.498751) < 1e-6
    assert abs(r.prob(2, 1) - 0.749178) < 1e-6
    r.close()


def test_inits(env):
    r = qa.Register(env, 4)
    r.init_plus()
    assert np.allclose(r.to_numpy(), np.full(16, 0.25))
    r.init_classical(5)
    v = np.zeros(16)
    v[5] = 1
    assert np.allclose(r.to_numpy(), v)
    r.init_debug()
    i = np.arange(16)
    assert np.allclose(r.to_numpy(), 0.2 * i + 1j * (0.2 * i + 0.1))
    r.close()
    d = qa.Register(env, 2, density=True)
    d.init_plus()
    assert np.allclose(d.to_numpy(), np.full((4, 4), 0.25))
    d.init_classical(2)
    m = np.zeros((4, 4))
    m[2, 2] = 1
    assert np.allclose(d.to_numpy(), m)
    d.close()


def test_init_single_qubit_and_pure(env, rng):
    from quest_amd.ops import capi
    from quest_amd.utils import oracle as O

    r = qa.Register(env, 4)
    capi.initStateOfSingleQubit(r.q, 2, 1)
    idx = np.arange(16)
    want = np.where((idx >> 2) & 1, 1 / np.sqrt(8), 0)
    assert np.allclose(r.to_numpy(), want)
    psi = O.random_state(rng, 4)
    r.set_amps(psi)
    d = qa.Register(env, 4, density=True)
    d.init_pure(r)
    assert np.allclose(d.to_numpy(), np.outer(psi, psi.conj()))
    assert abs(d.fidelity(r) - 1) < 1e-12
    assert abs(d.purity() - 1) < 1e-12
    r.close()
    d.close()
