"""One-pass marginals behind calcProbOfOutcome (router::probZero cache).

The fork's program asks for P(q = 1) of every qubit back to back
(/root/reference/tutorial_example.c:521-525).  The first query after a state
change reads one bit's half of the state; a second query of the same state
computes all marginals in one pass (be::marginals) and later queries come from
that cache until the next change.  These tests pin the values against the
NumPy oracle, the cache's invalidation on every kind of state change, and the
number of marginal passes."""
import numpy as np
import pytest

from helpers import apply_random_ops, load_state, oracle_for
from quest_amd.ops import capi
from quest_amd.utils import oracle as O


def _marg(v, n, q):
    p = np.abs(v.reshape([2] * n)) ** 2
    axes = tuple(n - 1 - k for k in range(n) if k != q)
    return p.sum(axis=axes)   # [P(q=0), P(q=1)]


def _stats():
    return capi.getQuESTStats()["marginalPasses"]


@pytest.mark.parametrize("n", [5, 13, 15])
def test_all_marginals_match_oracle(env, rng, n):
    import quest_amd as qa

    r = qa.Register(env, n)
    o = oracle_for(r, rng)
    apply_random_ops(r, o, rng, 60)
    before = _stats()
    for q in range(n):
        for outcome in (1, 0):
            assert r.prob(q, outcome) == pytest.approx(_marg(o.v, n, q)[outcome], abs=1e-12)
    assert _stats() - before == 1, "all 2n queries of one state: one marginal pass"
    r.close()


def test_cache_invalidated_by_every_state_change(env, rng):
    import quest_amd as qa

    n = 14
    r = qa.Register(env, n)
    o = oracle_for(r, rng)
    other = qa.Register(env, n)
    o2 = oracle_for(other, rng)

    def check():
        for q in (0, 7, n - 1):
            assert r.prob(q, 0) == pytest.approx(_marg(o.v, n, q)[0], abs=1e-12)
        assert r.total_prob() == pytest.approx(np.vdot(o.v, o.v).real, abs=1e-12)

    check()
    r.h(3)
    o.apply(O.H, 3)
    check()
    # collapse (non-unitary op)
    r.collapse(5, 1)
    o.collapse(5, 1)
    check()
    # overwrite paths
    load_state(r, o2.v)
    o.v = o2.v.copy()
    check()
    r.init_plus()
    o.v = np.full(1 << n, 1 / np.sqrt(1 << n), dtype=complex)
    check()
    capi.cloneQureg(r.q, other.q)
    o.v = o2.v.copy()
    check()
    # host buffers -> state
    import torch

    v = 1.5 * np.roll(o2.v, 3)     # unnormalised: the cached norm must change
    r.from_torch(torch.from_numpy(v))
    o.v = v
    check()
    r.close()
    other.close()


def test_interleaved_queries_and_gates(env, rng):
    """prob, gate, prob, ...: every query is answered for the current state."""
    import quest_amd as qa

    n = 13
    r = qa.Register(env, n)
    o = oracle_for(r, rng)
    for step in range(12):
        apply_random_ops(r, o, rng, 3)
        qs = rng.choice(n, size=3, replace=False)
        for q in qs:
            assert r.prob(int(q), 1) == pytest.approx(_marg(o.v, n, int(q))[1], abs=1e-12)
    r.close()


def test_density_probabilities_unaffected(env, rng):
    import quest_amd as qa

    r = qa.Register(env, 4, density=True)
    o = oracle_for(r, rng)
    apply_random_ops(r, o, rng, 20)
    for q in range(4):
        d = np.real(np.diag(o.rho)).reshape([2] * 4)
        axes = tuple(3 - k for k in range(4) if k != q)
        assert r.prob(q, 0) == pytest.approx(d.sum(axis=axes)[0], abs=1e-12)
    r.close()


def test_norm_cached_per_state(env, rng):
    """calcTotalProb reads the state once per state change (router::sumSqAll)."""
    import quest_amd as qa

    r = qa.Register(env, 12)
    o = oracle_for(r, rng)
    apply_random_ops(r, o, rng, 30)
    r.sync()
    before = capi.getQuESTStats()["reductions"]
    for _ in range(5):
        assert r.total_prob() == pytest.approx(1.0, abs=1e-12)
    assert capi.getQuESTStats()["reductions"] - before == 1
    r.x(2)
    o.apply(O.X, 2)
    r.total_prob()
    assert capi.getQuESTStats()["reductions"] - before == 2
    r.close()
