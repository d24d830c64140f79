"""Wave-engine planner knobs on the GPU.

Every combination of the load-layout order (``wave_lane_order`` 0/1/2) and the
XCD-aware tile order (``wave_tile_map`` 0/1) must give the same state as the
LDS tile kernel, and -- with the per-pass shadow check on -- every wave pass
must match the host emulation of the same plan (src/core/wave_emu.cpp), so a
kernel behaviour the emulator does not model shows up as the pass that
differs instead of as a wrong norm at the end.

Circuits: the 24-qubit layered circuit of test_checkpoint_round_trip_gpu
(where lane order 2 + tile map off once gave <psi|psi> = 1.0022) and a
30-qubit random_mixed circuit with two thirds of its gates on the top qubits.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_KNOBS = ("tile_mode", "wave_lane_order", "wave_tile_map", "wave_shadow", "wave_wg_per_cu")


@pytest.fixture(scope="module")
def genv():
    import quest_amd as qa

    e = qa.Env()
    assert qa.capi.getQuESTBackend() == "HIP"
    return e


@pytest.fixture(autouse=True)
def restore(genv):
    from quest_amd.ops import capi

    saved = {k: capi.getQuESTTuning(k) for k in _KNOBS}
    yield
    for k, v in saved.items():
        capi.setQuESTTuning(k, v)


def _run(genv, n, circ, knobs):
    import quest_amd as qa
    from quest_amd.ops import capi

    for k, v in knobs.items():
        assert capi.setQuESTTuning(k, v) == 1, k
    r = qa.Register(genv, n)
    r.init_plus()
    capi.resetQuESTStats()
    circ.apply(r)
    r.sync()
    st = capi.getQuESTStats()
    return r, st


@pytest.mark.parametrize("depth", [2, 6])
@pytest.mark.parametrize("grid", [0, 3])
@pytest.mark.parametrize("tile_map", [0, 1])
@pytest.mark.parametrize("lane_order", [0, 1, 2])
def test_lane_order_tile_map_24q(genv, lane_order, tile_map, grid, depth):
    """grid 0: one workgroup per tile (default); 3: a persistent grid of three
    workgroups per CU looping over the tiles (the tile map needs it)."""
    from quest_amd.models import random_layered

    n = 24
    circ = random_layered(n, depth, seed=2)
    ref, _ = _run(genv, n, circ, {"tile_mode": 0, "wave_shadow": 0})
    a, st = _run(genv, n, circ, {"tile_mode": 3, "wave_lane_order": lane_order, "wave_tile_map": tile_map,
                                 "wave_wg_per_cu": grid, "wave_shadow": 1})
    assert st["wavePasses"] > 0, st
    assert st["waveShadowChecks"] == st["wavePasses"], st
    assert st["waveShadowMismatches"] == 0, st
    # the shadow check repairs a bad pass: compare with the shadow off too
    b, st2 = _run(genv, n, circ, {"tile_mode": 3, "wave_lane_order": lane_order, "wave_tile_map": tile_map,
                                  "wave_wg_per_cu": grid, "wave_shadow": 0})
    want = ref.to_numpy()
    for r in (a, b):
        got = r.to_numpy()
        assert np.max(np.abs(got - want)) < 1e-12
        assert abs(r.total_prob() - 1) < 1e-12
    for r in (ref, a, b):
        r.close()


@pytest.mark.parametrize("tile_map", [0, 1])
@pytest.mark.parametrize("lane_order", [0, 1, 2])
def test_lane_order_tile_map_30q_mixed(genv, lane_order, tile_map):
    import quest_amd as qa
    from quest_amd.models import random_mixed

    n = 30
    circ = random_mixed(n, 300, seed=77 + lane_order, high=8)
    ref, _ = _run(genv, n, circ, {"tile_mode": 0, "wave_shadow": 0})
    a, st = _run(genv, n, circ, {"tile_mode": 3, "wave_lane_order": lane_order, "wave_tile_map": tile_map,
                                 "wave_shadow": 0})
    assert st["wavePasses"] > 0, st
    ov = a.inner(ref)
    assert 2 - 2 * ov.real < 1e-12, ov
    assert abs(a.total_prob() - 1) < 1e-11
    pa = np.array([a.prob(q, 1) for q in range(n)])
    pb = np.array([ref.prob(q, 1) for q in range(n)])
    np.testing.assert_allclose(pa, pb, rtol=0, atol=1e-12)
    a.close()
    ref.close()
    del qa
