"""GPU tests at the benchmark's scale, on the DEFAULT engine (fp64: the
wave-tile kernel): 30-qubit random circuits with controls and targets on the
top qubits against the LDS tile kernel, a 34-qubit (256 GiB) circuit followed
by its inverse, and the RCCL transport's code paths on a one-rank
communicator.  The golden cases are 3-qubit and never reach the wave engine
(it needs >= 19 local qubits), so these pin the shipped default at scale."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def genv():
    import quest_amd as qa

    e = qa.Env()
    assert qa.capi.getQuESTBackend() == "HIP"
    assert qa.capi.getQuESTTuning("tile_mode") == 3
    return e


def _run(reg, circ, tile_mode):
    import quest_amd as qa

    assert qa.capi.setQuESTTuning("tile_mode", tile_mode) == 1
    try:
        qa.capi.resetQuESTStats()
        circ.apply(reg)
        reg.sync()
        return qa.capi.getQuESTStats()
    finally:
        qa.capi.setQuESTTuning("tile_mode", 3)


@pytest.mark.parametrize("high", [0, 8])
def test_wave_engine_matches_lds_kernel_30q(genv, high):
    """600 mixed gates (controlled rotations, CY, multi-controlled Z, phases)
    on 30 qubits, two in three of them on the top `high` qubits: the wave
    engine and the LDS kernel must agree to 1e-12 in state overlap and in
    every single-qubit marginal."""
    import quest_amd as qa
    from quest_amd.models import random_mixed

    n = 30
    circ = random_mixed(n, 600, seed=30 + high, high=high)
    a = qa.Register(genv, n)
    b = qa.Register(genv, n)
    a.init_plus()
    b.init_plus()
    sa = _run(a, circ, 3)
    sb = _run(b, circ, 0)
    assert sa["wavePasses"] > 0 and sa["wavePasses"] >= sa["passes"] - 2, sa
    assert sb["wavePasses"] == 0, sb
    ov = a.inner(b)
    # |a - b|^2 = 2 - 2 Re<a|b>
    assert 2 - 2 * ov.real < 1e-12, ov
    assert abs(a.total_prob() - 1) < 1e-11
    pa = np.array([a.prob(q, 1) for q in range(n)])
    pb = np.array([b.prob(q, 1) for q in range(n)])
    np.testing.assert_allclose(pa, pb, rtol=0, atol=1e-12)
    for i in (0, 1, (1 << n) - 1, 123456789):
        assert abs(a.amp(i) - b.amp(i)) < 1e-12
    a.close()
    b.close()


def test_34_qubits_circuit_then_inverse(genv):
    """34 qubits (2^34 amplitudes, 256 GiB on one MI355X): a random layered
    circuit U followed by U^dagger must return |0...0> with amp(0) = 1 to
    1e-10, on the wave engine."""
    import quest_amd as qa
    from quest_amd.models import random_layered

    n = 34
    u = random_layered(n, 3, seed=34)
    r = qa.Register(genv, n)
    r.init_zero()
    qa.capi.resetQuESTStats()
    u.apply(r)
    p_mid = r.prob(n - 1, 1)
    assert 0 < p_mid < 1
    u.inverse().apply(r)
    r.sync()
    st = qa.capi.getQuESTStats()
    assert st["wavePasses"] > 0, st
    a0 = r.amp(0)
    assert abs(a0 - 1) < 1e-10, a0
    assert abs(r.total_prob() - 1) < 1e-10
    r.close()


def test_search_split_window_then_inverse(genv):
    """A 28-qubit, 10-layer window (~420 ops: below the front-flush
    threshold, above the strategy search's): the full flush launches its first
    pass at once and searches the rest while it runs (QUEST_PLAN_SEARCH_SPLIT,
    wave.cpp waveSearchSplitFirst); U then U^dagger, each such a window, must
    return |+...+> with every sampled amplitude 2^-14 to 1e-10."""
    import quest_amd as qa
    from quest_amd.models import random_layered

    n = 28
    u = random_layered(n, 10, seed=28)
    assert 256 < len(u.gates) < 600
    r = qa.Register(genv, n)
    r.init_plus()
    qa.capi.resetQuESTStats()
    u.apply(r)
    p_mid = r.prob(n // 2, 1)
    assert 0 < p_mid < 1
    u.inverse().apply(r)
    r.sync()
    st = qa.capi.getQuESTStats()
    # two windows, each split into its first pass's flush and the rest
    assert st["wavePasses"] > 0 and st["flushes"] >= 4, st
    want = 2.0 ** (-n / 2)
    for idx in (0, 1, 12345, (1 << n) - 1, 1 << 27, 987654321 % (1 << n)):
        a = r.amp(idx)
        assert abs(a - want) < 1e-10, (idx, a)
    assert abs(r.total_prob() - 1) < 1e-10
    r.close()


def test_rccl_transport_self_test(genv):
    """The RCCL transport's own calls on hardware: a one-rank communicator
    runs the pipelined exchange (communication stream + events, 5 slices over
    2 buffer sets, grouped send/recv), the staged scalar allreduce and
    broadcast, allgather and the async-error poll (quest_amd.h
    runCommSelfTest)."""
    from quest_amd.ops import capi

    ok, report = capi.runCommSelfTest()
    assert ok, report
    assert "RCCL" in report and "WRONG" not in report, report
    print(report)


def test_one_pass_marginals_26q(genv):
    """Every qubit's marginal from the one-pass kernel (second query of a
    state fills the cache) against marginals computed by torch from the
    state itself, on 26 qubits (2^14 tiles, 11 workgroup bits, 3 varying tile
    bits)."""
    import torch

    import quest_amd as qa
    from quest_amd.models import random_layered

    n = 26
    r = qa.Register(genv, n)
    r.init_plus()
    random_layered(n, 4, seed=26).apply(r)
    before = qa.capi.getQuESTStats()["marginalPasses"]
    got = np.array([r.prob(q, 0) for q in range(n)])
    assert qa.capi.getQuESTStats()["marginalPasses"] - before == 1
    p = (r.to_torch().abs() ** 2).reshape([2] * n)
    want = np.array([float(p.sum(dim=tuple(n - 1 - k for k in range(n) if k != q))[0]) for q in range(n)])
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-12)
    r.close()


@pytest.mark.parametrize("mode", [None, "0", "1", "2", "3"])
def test_register_placements_agree_27q(genv, mode, monkeypatch):
    """Every placement of a register's arrays (default: one allocation with
    an 8 GiB gap between re and im; 0 two allocations; 1 joint; 2 physically
    contiguous; 3 reserved address range with mapped arrays) gives the same
    state bit for bit on a 27-qubit circuit (1 GiB arrays: the default takes
    its gap), including amplitude reads and writes and a clone."""
    import quest_amd as qa
    from quest_amd.models import random_layered

    if mode is None:
        monkeypatch.delenv("QUEST_ALLOC_MODE", raising=False)
    else:
        monkeypatch.setenv("QUEST_ALLOC_MODE", mode)
        monkeypatch.setenv("QUEST_IM_OFFSET", str(1 << 30))
        monkeypatch.setenv("QUEST_IM_DIST", str(3 << 30))
    n = 27
    circ = random_layered(n, 3, seed=27)
    r = qa.Register(genv, n)
    monkeypatch.delenv("QUEST_ALLOC_MODE", raising=False)
    ref = qa.Register(genv, n)          # default placement
    for reg in (r, ref):
        reg.init_plus()
        circ.apply(reg)
        reg.set_amps(np.array([0.25 + 0.5j, -0.125j]), start=5)
        reg.h(0)
    idx = [0, 1, 5, 6, 12345, (1 << n) - 1]
    got = [r.amp(i) for i in idx]
    want = [ref.amp(i) for i in idx]
    assert got == want
    assert 2 - 2 * r.inner(ref).real < 1e-13
    c = qa.Register(genv, n)
    c.clone_from(r)
    assert c.amp(12345) == r.amp(12345)
    for reg in (r, ref, c):
        reg.close()
