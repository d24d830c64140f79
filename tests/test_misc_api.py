"""The remaining API surface: reporting (reportState CSV, reportStateToScreen,
reportQuregParams, reportQuESTEnv, getEnvironmentString), file input
(initStateFromSingleFile), debug helpers (compareStates,
initStateOfSingleQubit, initStateDebug on density matrices), seeding, and the
MI355X extensions (statistics, layout, chunk buffers, fusion switch)."""
import os

import numpy as np
import pytest

from quest_amd.ops import capi


def test_report_state_csv(env, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    q = capi.createQureg(2, env.env)
    capi.initStateDebug(q)
    capi.reportState(q)
    text = (tmp_path / "state_rank_0.csv").read_text()
    assert text == ("real, imag\n0.000000000000, 0.100000000000\n0.200000000000, 0.300000000000\n"
                    "0.400000000000, 0.500000000000\n0.600000000000, 0.700000000000\n")
    capi.destroyQureg(q, env.env)


def test_init_state_from_single_file(env, tmp_path):
    path = tmp_path / "amps.csv"
    path.write_text("# comment lines are skipped\n0.5, 0.0\n0.0, 0.5\n# another\n-0.5, 0.0\n0.0, -0.5\n")
    q = capi.createQureg(2, env.env)
    capi.initStateFromSingleFile(q, str(path), env.env)
    np.testing.assert_allclose(capi.getAmps(q), [0.5, 0.5j, -0.5, -0.5j])
    capi.destroyQureg(q, env.env)


def test_compare_states_and_single_qubit_init(env):
    a, b = capi.createQureg(4, env.env), capi.createQureg(4, env.env)
    capi.initStateOfSingleQubit(a, 2, 1)
    v = capi.getAmps(a)
    idx = np.arange(16)
    np.testing.assert_allclose(v, np.where((idx >> 2) & 1, 1 / np.sqrt(8), 0))
    capi.cloneQureg(b, a)
    assert capi.compareStates(a, b, 1e-12) == 1
    capi.rotateX(b, 0, 1e-3)
    assert capi.compareStates(a, b, 1e-12) == 0
    assert capi.compareStates(a, b, 1e-2) == 1
    capi.destroyQureg(a, env.env)
    capi.destroyQureg(b, env.env)


def test_report_params_env_and_strings(env, capfd):
    q = capi.createQureg(5, env.env)
    d = capi.createDensityQureg(3, env.env)
    capi.reportQuregParams(q)
    out = capfd.readouterr().out
    assert out == "QUBITS:\nNumber of qubits is 5.\nNumber of amps is 32.\nNumber of amps per rank is 32.\n"
    capi.reportQuregParams(d)
    assert "Number of qubits is 6." in capfd.readouterr().out
    capi.reportQuESTEnv(env.env)
    out = capfd.readouterr().out
    assert out.startswith("EXECUTION ENVIRONMENT:\n") and "Number of ranks is 1" in out
    s = capi.getEnvironmentString(env.env, q)
    assert s == f"5qubits_{capi.getQuESTBackend()}_1ranks"
    assert capi.getNumQubits(d) == 3 and capi.getNumAmps(q) == 32
    capi.destroyQureg(q, env.env)
    capi.destroyQureg(d, env.env)


def test_density_debug_state_and_amps(env):
    d = capi.createDensityQureg(2, env.env)
    capi.initStateDebug(d)
    flat = capi.getAmps(d)
    k = np.arange(16)
    np.testing.assert_allclose(flat, 0.2 * k + 1j * (0.2 * k + 0.1))
    # element (r, c) lives at r + c * 2^n
    assert capi.getDensityAmp(d, 1, 2) == pytest.approx(flat[1 + 2 * 4])
    capi.destroyQureg(d, env.env)


def test_seeds_roundtrip(env):
    import ctypes as C

    b = capi.binding()
    capi.seedQuEST([5, 6, 7])
    arr = (C.c_ulong * 64)()
    n = C.c_int(0)
    b.lib.getQuESTSeeds(arr, C.byref(n))
    assert n.value == 3 and list(arr[:3]) == [5, 6, 7]
    capi.seedQuEST([5, 6, 7])
    x = [capi.genrand_real1() for _ in range(3)]
    capi.seedQuEST([5, 6, 7])
    assert [capi.genrand_real1() for _ in range(3)] == x
    capi.seedQuESTDefault()
    b.lib.getQuESTSeeds(arr, C.byref(n))
    assert n.value == 2


def test_get_prob_amp_and_real_imag(env):
    q = capi.createQureg(3, env.env)
    capi.initStateDebug(q)
    assert capi.getRealAmp(q, 5) == pytest.approx(1.0)
    assert capi.getImagAmp(q, 5) == pytest.approx(1.1)
    assert capi.getProbAmp(q, 5) == pytest.approx(1.0 + 1.21)
    capi.destroyQureg(q, env.env)


def test_stats_layout_and_fusion_switch(env):
    import quest_amd as qa
    from quest_amd.models import random_layered

    c = random_layered(12, 3, seed=4)
    outs = []
    for fuse in (1, 0):
        capi.setGateFusion(fuse)
        assert capi.getGateFusion() == fuse
        r = qa.Register(env, 12)
        r.init_plus()
        capi.resetQuESTStats()
        c.apply(r)
        r.sync()
        st = capi.getQuESTStats()
        assert st["opsQueued"] >= len(c.gates)
        if fuse:
            assert st["passes"] < len(c.gates)
        else:
            assert st["passes"] >= len(c.gates)
        assert capi.getQubitLayout(r.q) == list(range(12))
        outs.append(r.to_numpy())
        r.close()
    capi.setGateFusion(1)
    np.testing.assert_allclose(outs[0], outs[1], atol=1e-12)


def test_chunk_buffers_host_build(env):
    if capi.getQuESTBackend() != "CPU":
        pytest.skip("host-buffer variant; the GPU test uses torch tensors")
    b = capi.binding()
    q = capi.createQureg(4, env.env)
    capi.initStateDebug(q)
    re = np.zeros(16)
    im = np.zeros(16)
    capi._call("copyChunkToBuffers", q, re.ctypes.data, im.ctypes.data)
    np.testing.assert_allclose(re + 1j * im, capi.getAmps(q))
    re2, im2 = 2 * re, 2 * im  # keep the arrays alive across the call
    capi._call("copyChunkFromBuffers", q, re2.ctypes.data, im2.ctypes.data)
    np.testing.assert_allclose(capi.getAmps(q), 2 * (re + 1j * im))
    capi.destroyQureg(q, env.env)
    assert b.backend == "cpu"


def test_init_pure_and_add_density(env):
    from quest_amd.utils import oracle as O

    rng = np.random.default_rng(3)
    psi = O.random_state(rng, 3)
    p = capi.createQureg(3, env.env)
    capi.setAmps(p, 0, psi.real, psi.imag, 8)
    d = capi.createDensityQureg(3, env.env)
    capi.initPureState(d, p)
    rho = np.outer(psi, psi.conj())
    got = capi.getAmps(d).reshape(8, 8, order="F")
    np.testing.assert_allclose(got, rho, atol=1e-12)
    assert capi.calcFidelity(d, p) == pytest.approx(1.0, abs=1e-12)
    d2 = capi.createDensityQureg(3, env.env)
    capi.initClassicalState(d2, 6)
    capi.addDensityMatrix(d, 0.25, d2)
    want = 0.75 * rho
    want[6, 6] += 0.25
    np.testing.assert_allclose(capi.getAmps(d).reshape(8, 8, order="F"), want, atol=1e-12)
    for r in (p, d, d2):
        capi.destroyQureg(r, env.env)


def test_host_state_edit_then_copy_to_gpu_refreshes_caches(env):
    """The reference idiom: write qureg.stateVec directly, then
    copyStateToGPU.  On the host build stateVec is the live state; the cached
    norm / marginals must not survive the edit."""
    q = capi.createQureg(3, env.env)
    capi.initPlusState(q)
    assert abs(capi.calcTotalProb(q) - 1) < 1e-12
    p0 = capi.calcProbOfOutcome(q, 0, 0)
    assert abs(p0 - 0.5) < 1e-12
    re = q.stateVec.real
    for i in range(8):
        re[i] = 1.0 if i == 0 else 0.0
        q.stateVec.imag[i] = 0.0
    capi.copyStateToGPU(q)
    assert abs(capi.calcTotalProb(q) - 1) < 1e-12
    assert abs(capi.calcProbOfOutcome(q, 0, 0) - 1) < 1e-12
    re[0] = 0.0
    re[1] = 2.0 ** -0.5
    re[3] = 2.0 ** -0.5
    capi.copyStateToGPU(q)
    assert abs(capi.calcProbOfOutcome(q, 0, 1) - 1) < 1e-12
    assert abs(capi.calcProbOfOutcome(q, 1, 1) - 0.5) < 1e-12
    capi.destroyQureg(q, env.env)
