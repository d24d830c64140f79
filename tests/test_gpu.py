"""HIP (gfx950) backend tests: every kernel family against the NumPy oracle
(fp32/fp64 reference computations of the same ops), at qubit counts that
exercise every tile geometry (whole-state tile, multi-tile, high targets,
controls outside the tile) and the fused / unfused paths."""
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def genv():
    import quest_amd as qa

    e = qa.Env()
    assert qa.capi.getQuESTBackend() == "HIP", "HIP library not loaded on a GPU test run"
    return e


_KNOBS = ("tile_mode", "direct_kernels", "tile_qubits", "direct_layout", "direct_low_to_tile", "tile_wg_per_cu",
          "wave_wg_per_cu", "fuse_blocks", "verify", "wave_lane_order", "wave_tile_map", "wave_shadow")


@pytest.fixture(autouse=True)
def restore_tuning(genv):
    """Every test leaves the engine configuration as it found it -- the
    build's defaults (fp64: the wave-tile engine, tile_mode 3) -- whatever
    it changed (round 1 restored tile_mode 0 and silently ran the rest of
    the module on the LDS kernel)."""
    from quest_amd.ops import capi

    saved = {k: capi.getQuESTTuning(k) for k in _KNOBS}
    fusion = capi.getGateFusion()
    yield
    for k, v in saved.items():
        if v is not None:
            capi.setQuESTTuning(k, v)
    capi.setGateFusion(fusion)
    capi.setFusionMaxQubits(0)


def test_wave_engine_is_the_fp64_default(genv):
    from quest_amd.ops import capi

    assert capi.getQuESTTuning("tile_mode") == 3
    assert capi.getQuESTTuning("direct_kernels") == 1


def test_native_hip_library_loaded(genv):
    from quest_amd.ops import capi

    b = capi.binding()
    assert b.backend == "hip"
    assert b.lib._quest_path.endswith("libQuEST_hip_f64.so")
    maps = open("/proc/self/maps").read()
    assert "libQuEST_hip_f64.so" in maps


@pytest.mark.parametrize("n", [3, 6, 9, 12, 15])
def test_all_gates_vs_oracle(genv, n):
    import quest_amd as qa
    from helpers import GATES_1Q, GATES_2Q, apply_named, assert_close, oracle_for

    rng = np.random.default_rng(n)
    reg = qa.Register(genv, n)
    for name in GATES_1Q:
        for t in range(n):
            o = oracle_for(reg, rng)
            apply_named(reg, o, name, [t], rng)
            assert_close(reg, o)
    for name in GATES_2Q:
        for _ in range(6):
            qs = [int(x) for x in rng.permutation(n)[:2]]
            o = oracle_for(reg, rng)
            apply_named(reg, o, name, qs, rng)
            assert_close(reg, o)
    for name in ("mcunitary", "mcphase", "mcz"):
        for k in range(2, min(n, 5) + 1):
            qs = [int(x) for x in rng.permutation(n)[:k]]
            o = oracle_for(reg, rng)
            apply_named(reg, o, name, qs, rng)
            assert_close(reg, o)
    reg.close()


@pytest.mark.parametrize("n", [3, 5, 7, 10])
def test_density_gates_and_noise(genv, n):
    """n = 10 (2^20 amplitudes): the wave engine runs the gates and the LDS
    kernel the channels, flushed as alternating runs of the mixed queue."""
    import quest_amd as qa
    from helpers import apply_random_ops, assert_close, oracle_for

    rng = np.random.default_rng(100 + n)
    reg = qa.Register(genv, n, density=True)
    for _ in range(3):
        o = oracle_for(reg, rng)
        apply_random_ops(reg, o, rng, 40, noise=True)
        assert_close(reg, o, tol=1e-9)
        assert abs(reg.total_prob() - np.real(np.trace(o.rho))) < 1e-10
        assert abs(reg.purity() - o.purity()) < 1e-10
        for q in range(n):
            assert abs(reg.prob(q, 0) - o.prob(q, 0)) < 1e-10
    reg.close()


@pytest.mark.parametrize("n", [10])
def test_density_one_qubit_channels_on_wave_engine(genv, n):
    """A density matrix of 10 qubits (2^20 amplitudes, the smallest the wave
    engine takes; the dense NumPy oracle is too slow beyond) under
    gates and one-qubit dephasing, depolarising and damping: every pass runs
    on the wave engine (channels as CH1 / CHD register ops on the row and
    column bits), against the NumPy oracle."""
    import quest_amd as qa
    from helpers import apply_random_ops, assert_close, oracle_for
    from quest_amd.utils import oracle as O

    rng = np.random.default_rng(300 + n)
    reg = qa.Register(genv, n, density=True)
    o = oracle_for(reg, rng)
    qa.capi.resetQuESTStats()
    apply_random_ops(reg, o, rng, 30)
    for k in range(40):
        a = int(rng.integers(n))
        p = float(rng.uniform(0, 0.5))
        [(reg.dephase, o.dephase), (reg.depolarise, o.depolarise), (reg.damping, o.damping)][k % 3][0](a, p)
        [(reg.dephase, o.dephase), (reg.depolarise, o.depolarise), (reg.damping, o.damping)][k % 3][1](a, p)
        if k % 5 == 0:
            reg.h(a)
            o.apply(O.H, a)
    reg.sync()
    st = qa.capi.getQuESTStats()
    assert st["wavePasses"] > 0 and st["wavePasses"] == st["passes"], st
    assert_close(reg, o, tol=1e-9)
    assert abs(reg.purity() - o.purity()) < 1e-10
    for q in range(n):
        assert abs(reg.prob(q, 0) - o.prob(q, 0)) < 1e-10
    reg.close()


@pytest.mark.parametrize("fusion", [True, False])
@pytest.mark.parametrize("n", [14, 20])
def test_random_circuit_fused_and_eager(genv, n, fusion):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.utils import oracle as O

    qa.capi.setGateFusion(1 if fusion else 0)
    c = random_layered(n, 3, seed=n)
    reg = qa.Register(genv, n)
    reg.init_plus()
    c.apply(reg)
    o = O.StateVector(n, np.full(1 << n, 1 / math.sqrt(1 << n)))
    c.apply_oracle(o)
    got = reg.to_numpy()
    assert np.max(np.abs(got - o.v)) < 1e-10
    for q in (0, n // 2, n - 1):
        assert abs(reg.prob(q, 1) - o.prob(q, 1)) < 1e-10
    reg.close()


@pytest.mark.parametrize("tile_mode", [0, 1, 2, 3])
@pytest.mark.parametrize("direct", [0, 1])
def test_long_queue_every_tile_mode(genv, tile_mode, direct):
    """More ops than one flush holds: 40 layers at 19 qubits are 1120 gates,
    so the 1024-op backend queue flushes itself mid-circuit, in every
    fused-tile variant (3 = the wave engine, which needs >= 19 local qubits);
    state must match the oracle."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.utils import oracle as O

    n = 19
    assert qa.capi.setQuESTTuning("tile_mode", tile_mode) == 1
    assert qa.capi.setQuESTTuning("direct_kernels", direct) == 1
    c = random_layered(n, 40, seed=tile_mode * 2 + direct)
    assert len(c.gates) > 1024
    reg = qa.Register(genv, n)
    reg.init_plus()
    qa.capi.resetQuESTStats()
    c.apply(reg)
    reg.sync()
    st = qa.capi.getQuESTStats()
    assert st["flushes"] >= 2, st
    if tile_mode == 3:
        assert st["wavePasses"] > 0, st
    o = O.StateVector(n, np.full(1 << n, 1 / math.sqrt(1 << n)))
    c.apply_oracle(o)
    assert np.max(np.abs(reg.to_numpy() - o.v)) < 1e-10
    reg.close()


def test_reductions_and_collapse_large(genv):
    """24 qubits: 128 MiB per array; norm, per-qubit probabilities, inner
    product and collapse against quantities computed from the same state."""
    import quest_amd as qa
    from quest_amd.models import random_layered

    n = 24
    a = qa.Register(genv, n)
    b = qa.Register(genv, n)
    a.init_plus()
    random_layered(n, 2, seed=3).apply(a)
    b.clone_from(a)
    assert abs(a.total_prob() - 1) < 1e-11
    ip = a.inner(b)
    assert abs(ip - 1) < 1e-11
    v = a.to_numpy()
    idx = np.arange(1 << n)
    for q in (0, 1, 5, 12, 23):
        want = float(np.sum(np.abs(v[((idx >> q) & 1) == 0]) ** 2))
        assert abs(a.prob(q, 0) - want) < 1e-11
    p = a.collapse(7, 1)
    assert abs(a.total_prob() - 1) < 1e-11
    assert a.prob(7, 1) > 1 - 1e-11
    assert p > 0
    a.close()
    b.close()


def test_measure_seeded_matches_cpu_semantics(genv):
    """Seeded measurement reproduces the reference's expectations
    (tests/unit/state_vector/maths/measure.test:11-45)."""
    import quest_amd as qa
    from quest_amd.ops import capi

    q = qa.Register(genv, 3)
    q.init_zero()
    capi.seedQuEST([1])
    assert [q.measure(i) for i in range(3)] == [0, 0, 0]
    q.init_plus()
    assert [q.measure(i) for i in range(3)] == [0, 1, 1]
    q.close()


def test_torch_interop(genv):
    import torch

    import quest_amd as qa

    r = qa.Register(genv, 10)
    r.init_debug()
    t = r.to_torch()
    i = torch.arange(1 << 10, device="cuda", dtype=torch.float64)
    assert torch.allclose(t.real, 0.2 * i) and torch.allclose(t.imag, 0.2 * i + 0.1)
    r.from_torch(t * 2)
    assert abs(r.amp(3) - 2 * (0.6 + 0.7j)) < 1e-12
    r.close()


def test_fusion_reduces_passes(genv):
    import quest_amd as qa
    from quest_amd.models import random_layered

    n = 22
    c = random_layered(n, 4, seed=11)
    reg = qa.Register(genv, n)
    reg.init_plus()
    qa.capi.resetQuESTStats()
    c.apply(reg)
    reg.sync()
    st = qa.capi.getQuESTStats()
    assert st["passes"] < len(c.gates) / 4, st
    assert abs(reg.total_prob() - 1) < 1e-10
    reg.close()


def test_fp32_library_builds_and_loads():
    """The fp32 HIP library is a separate compile-time build (QuEST_PREC=1);
    check it in a subprocess (a process binds one precision)."""
    import subprocess
    import sys

    code = (
        "import quest_amd as qa, math\n"
        "e = qa.Env(); r = qa.Register(e, 12); r.init_plus(); r.h(3); r.rx(7, 0.3); r.cnot(2, 9)\n"
        "assert abs(r.total_prob() - 1) < 1e-5\n"
        "from quest_amd.ops import capi; assert capi.getQuEST_PREC() == 1\n"
        "print('fp32 ok')\n"
    )
    envv = dict(os.environ, QUEST_PREC="1", QUEST_BACKEND="hip")
    out = subprocess.run([sys.executable, "-c", code], env=envv, capture_output=True, text=True, timeout=300,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    assert "fp32 ok" in out.stdout


def test_reference_golden_suite_on_gpu(genv):
    """All golden cases of the reference's tests/**/*.test data on the HIP
    backend (tests/test_reference_suite.py runs them on the CPU build)."""
    from quest_amd.utils import golden

    passed, failures = golden.run_all(genv.env)
    assert not failures, "\n".join(failures[:20])
    assert passed >= 770


_DIST = ["random_ops_statevector", "random_ops_density", "measurement_and_collapse", "calculations", "qasm_log",
         "rank_qubit_gates", "top_swap", "restore_chunks"]


@pytest.mark.parametrize("transport,ranks,slice_kb", [("ipc", 2, ""), ("ipc", 4, ""), ("ipc-buffered", 4, "1"),
                                                      ("ipc-nopipe", 2, "1"), ("socket", 2, ""), ("rccl", 2, ""),
                                                      ("rccl", 4, "1")])
@pytest.mark.parametrize("name", _DIST)
def test_distributed_equivalence_on_gpu(genv, tmp_path, name, transport, ranks, slice_kb):
    """The distributed router with the HIP kernels (pack/unpack, chunk
    predicates, reductions + allreduce) on ONE GPU shared by 2 / 4 ranks,
    against the single-rank HIP run.  QUEST_COMM=ipc swaps parts in place
    (one kernel per rank pair through the peer's mapped state);
    ipc-buffered (QUEST_IPC_SWAP=0) moves the slices GPU-to-GPU-buffer
    through HIP IPC on the communication stream with the RCCL transport's
    event protocol (pack / exchange / unpack overlapped, double-buffered);
    ipc-nopipe runs every buffered exchange on the compute stream
    (QUEST_EXCHANGE_PIPELINE=0); socket stages through the host; rccl runs
    the production RCCL calls (grouped send / recv on the communication
    stream, allreduce, broadcast) with N ranks on the one GPU
    (QUEST_RCCL_SHARED_GPU=1: RCCL's network transport over loopback).
    slice_kb=1 splits every swap into many double-buffered slices."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from scenarios import SCENARIOS

    from quest_amd.parallel import spawn_local

    want = SCENARIOS[name](genv)
    out = str(tmp_path / f"{name}_{ranks}.npz")
    extra = {"QUEST_BACKEND": "hip", "QUEST_COMM": transport.split("-")[0], "PYTHONPATH": os.path.dirname(here),
             "QUEST_COMM_TIMEOUT": "180"}
    if transport == "ipc-nopipe":
        extra.update(QUEST_EXCHANGE_PIPELINE="0", QUEST_IPC_SWAP="0")
    if transport == "ipc-buffered":
        extra["QUEST_IPC_SWAP"] = "0"
    if transport == "rccl":
        # a rank that hangs dumps its Python stack and exits (QUEST_TEST_STACKS)
        extra.update(QUEST_RCCL_SHARED_GPU="1", QUEST_COMM_TIMEOUT="60", QUEST_TEST_STACKS="120")
    if slice_kb:
        extra["QUEST_EXCHANGE_SLICE_KB"] = slice_kb
    res = spawn_local([os.path.join(here, "dist_worker.py"), name, out], ranks, env_extra=extra, timeout=200)
    # every rank's output on failure: the first rank's error is often only
    # "peer closed the connection" from another rank that failed first
    bad = [(r, p) for r, p in enumerate(res) if p.returncode != 0]
    assert not bad, "\n".join(f"rank {r} (rc {p.returncode}):\n{p.stdout[-1500:]}\n{p.stderr[-2500:]}" for r, p in bad)
    with np.load(out, allow_pickle=False) as z:
        got = {k: z[k] for k in z.files}
    assert int(got["_ranks"]) == ranks
    assert {"ipc": "IPC", "socket": "socket", "rccl": "RCCL"}[transport.split("-")[0]] in str(got["_transport"])
    for k, v in want.items():
        if k.startswith("_"):
            continue  # per-run statistics (swaps, restore rounds) depend on the rank count
        if isinstance(v, str):
            assert str(got[k]) == v, k
        else:
            np.testing.assert_allclose(np.asarray(got[k]), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)
    if name == "restore_chunks":
        # one concurrent round moving one chunk per rank (in place over IPC)
        assert int(got["_xor_rounds"]) == 1
        assert int(got["_xor_bytes"]) == 16 * (1 << (9 - {2: 1, 4: 2}[ranks]))


@pytest.mark.parametrize("transport", ["ipc", "rccl"])
def test_rank_controlled_relabel_layouts_on_gpu(genv, tmp_path, monkeypatch, transport):
    """Wave-sized ranks (4 x 22 local qubits on one GPU) whose planners see
    different op lists -- CNOTs controlled by rank qubits run only where the
    bit is 1 -- and so relabel differently: every swap first aligns the
    ranks' local layouts (router alignLayouts).  The in-place IPC swap, which
    indexes the peer's state with its own layout, lost norm (1e-5 .. 3e-3 on
    the bench's seeds 13 / 17 at 8 ranks) before; the buffered paths were off
    by a permutation.  Against the single-rank HIP run."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from scenarios import SCENARIOS

    from quest_amd.parallel import spawn_local

    monkeypatch.setenv("RCR_QUBITS", "24")
    want = SCENARIOS["rank_controlled_relabel"](genv)
    out = str(tmp_path / "rcr.npz")
    extra = {"QUEST_BACKEND": "hip", "QUEST_COMM": transport, "PYTHONPATH": os.path.dirname(here),
             "QUEST_COMM_TIMEOUT": "120", "RCR_QUBITS": "24"}
    if transport == "rccl":
        extra["QUEST_RCCL_SHARED_GPU"] = "1"
    res = spawn_local([os.path.join(here, "dist_worker.py"), "rank_controlled_relabel", out], 4, env_extra=extra,
                      timeout=200)
    bad = [(r, p) for r, p in enumerate(res) if p.returncode != 0]
    assert not bad, "\n".join(f"rank {r} (rc {p.returncode}):\n{p.stdout[-1500:]}\n{p.stderr[-2500:]}" for r, p in bad)
    with np.load(out, allow_pickle=False) as z:
        got = {k: z[k] for k in z.files}
    for k in ("probs", "amps", "norm"):
        np.testing.assert_allclose(np.asarray(got[k]), np.asarray(want[k]), rtol=0, atol=1e-11, err_msg=k)
    assert int(got["_swaps"]) > 0


IPC_F32 = r'''
import json, os, sys
import numpy as np
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi
env = qa.Env()
n = 18
r = qa.Register(env, n)
r.init_plus()
random_layered(n, 12, seed=5).apply(r)
r.x(n - 1)                 # chunk relabel, then restored by the read
r.ry(n - 2, 0.4)
v = r.to_numpy()
st = capi.getQuESTStats()
if env.rank == 0:
    np.save(sys.argv[1], v)
    print("STATS " + json.dumps({"swaps": st["swaps"], "ranks": env.num_ranks, "transport": capi.getQuESTTransport()}))
'''


@pytest.mark.parametrize("ranks", [2, 4])
def test_ipc_in_place_swaps_fp32(genv, tmp_path, ranks):
    """The fp32 library over the IPC transport: in-place part swaps
    (swapPartsKernel on float vectors) and chunk restores against one rank."""
    from quest_amd.parallel import spawn_local

    here = os.path.dirname(os.path.abspath(__file__))
    one, dist = str(tmp_path / "one.npy"), str(tmp_path / "dist.npy")
    base = {"QUEST_BACKEND": "hip", "QUEST_PREC": "1", "PYTHONPATH": os.path.dirname(here)}
    import subprocess
    import sys

    p = subprocess.run([sys.executable, "-c", IPC_F32, one], env=dict(os.environ, **base), capture_output=True,
                       text=True, timeout=200)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    res = spawn_local(["-c", IPC_F32, dist], ranks, env_extra=dict(base, QUEST_COMM="ipc", QUEST_COMM_TIMEOUT="120"),
                      timeout=200)
    for r, q in enumerate(res):
        assert q.returncode == 0, f"rank {r}:\n{q.stdout[-1500:]}\n{q.stderr[-2500:]}"
    st = json.loads([ln for ln in res[0].stdout.splitlines() if ln.startswith("STATS")][0][6:])
    assert st["ranks"] == ranks and "IPC" in st["transport"] and st["swaps"] >= 1, st
    a, b = np.load(one), np.load(dist)
    assert np.max(np.abs(a - b)) < 2e-6


IPC_RELEASE = r'''
import json, sys
import torch
import quest_amd as qa
from quest_amd.ops import capi
env = qa.Env()
torch.cuda.init()
env.sync()
free0 = torch.cuda.mem_get_info()[0]
frees = []
for it in range(3):
    r = qa.Register(env, 31)          # 16 GiB per rank, both ranks on this device
    r.init_plus()
    for q in range(31):
        r.h(q)                         # the top qubit is the rank qubit: a swap
    r.cnot(30, 0)
    assert abs(r.total_prob() - 1) < 1e-9
    r.close()
    env.sync()
    frees.append(torch.cuda.mem_get_info()[0])
st = capi.getQuESTStats()
if env.rank == 0:
    print("STATS " + json.dumps({"free0": free0, "frees": frees, "swaps": st["swaps"]}))
'''


def test_ipc_state_mappings_released_after_swaps(genv, tmp_path):
    """In-place IPC swaps map the peer's whole state; the mappings are closed
    when the swap completes (comm_ipc.cpp done()), so a destroyed register's
    memory returns to the device at once and destroy / create loops at large
    sizes do not accumulate pinned allocations (round-4 advisor finding)."""
    from quest_amd.parallel import spawn_local

    here = os.path.dirname(os.path.abspath(__file__))
    base = {"QUEST_BACKEND": "hip", "PYTHONPATH": os.path.dirname(here)}
    res = spawn_local(["-c", IPC_RELEASE], 2, env_extra=dict(base, QUEST_COMM="ipc", QUEST_COMM_TIMEOUT="120"),
                      timeout=240)
    for r, q in enumerate(res):
        assert q.returncode == 0, f"rank {r}:\n{q.stdout[-1500:]}\n{q.stderr[-2500:]}"
    st = json.loads([ln for ln in res[0].stdout.splitlines() if ln.startswith("STATS")][0][6:])
    assert st["swaps"] >= 3, st
    gib = 1 << 30
    # each 16 GiB chunk (32 GiB of states over both ranks) is back after every destroy
    for f in st["frees"]:
        assert f > st["free0"] - 3 * gib, st


OVERLAP = r'''
import json, sys
import numpy as np
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi
env = qa.Env()
n = int(sys.argv[2])
r = qa.Register(env, n)
r.init_plus()
capi.resetQuESTStats()
# a window whose ops before the swap leave local qubit hi alone and whose ops
# after it use hi last: hi is the victim, chosen before the pre-swap flush;
# the passes of that flush leave its position out of their tiles, so they run
# on the parts the swap sends first and on the part it keeps next to the transfer
top, hi = n - 1, 20
rng = np.random.default_rng(4)
for layer in range(6):
    for q in range(hi):
        r.ry(q, float(rng.uniform(0, 3)))
    for q in range(layer % 2, hi - 1, 2):
        r.cnot(q, q + 1)
r.h(top)
for q in range(hi + 1):
    r.cnot(top, q)
r.sync()
p = [r.prob(q, 1) for q in (0, hi, top)]
# a random layered circuit: its passes next to a swap always hold a swapped
# position (no split)
random_layered(n, 12, seed=3).apply(r)
r.sync()
st = capi.getQuESTStats()
v = r.to_numpy()
if env.rank == 0:
    np.save(sys.argv[1], v)
    print("STATS " + json.dumps({k: st[k] for k in ("swaps", "overlappedSwaps", "overlappedPasses")}))
'''


@pytest.mark.parametrize("ranks", [2, 4])
def test_overlapped_swaps_rccl_shared_gpu(genv, tmp_path, ranks):
    """Overlapped swaps (QUEST_SWAP_OVERLAP, default on): RCCL ranks sharing
    the GPU (QUEST_RCCL_SHARED_GPU=1, the RCCL path of a multi-GPU node) with
    21 local qubits.  A window whose ops before the swap leave the victim
    alone (its passes split: the parts the swap sends first, the kept part
    next to the transfer), then a random layered circuit (whose passes next to
    a swap always hold a swapped position: no split).  The state equals the
    single-rank run's and the split launches really happened."""
    from quest_amd.parallel import spawn_local

    here = os.path.dirname(os.path.abspath(__file__))
    n = 21 + {2: 1, 4: 2}[ranks]
    one, dist = str(tmp_path / "one.npy"), str(tmp_path / "dist.npy")
    base = {"QUEST_BACKEND": "hip", "PYTHONPATH": os.path.dirname(here)}
    import subprocess
    import sys

    p = subprocess.run([sys.executable, "-c", OVERLAP, one, str(n)], env=dict(os.environ, **base), capture_output=True,
                       text=True, timeout=200)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    res = spawn_local(["-c", OVERLAP, dist, str(n)], ranks,
                      env_extra=dict(base, QUEST_COMM="rccl", QUEST_RCCL_SHARED_GPU="1", QUEST_COMM_TIMEOUT="150"),
                      timeout=240)
    for r, q in enumerate(res):
        assert q.returncode == 0, f"rank {r}:\n{q.stdout[-1500:]}\n{q.stderr[-2500:]}"
    st = json.loads([ln for ln in res[0].stdout.splitlines() if ln.startswith("STATS")][0][6:])
    assert st["swaps"] >= 1 and st["overlappedSwaps"] >= 1 and st["overlappedPasses"] >= 1, st
    a, b = np.load(one), np.load(dist)
    assert np.max(np.abs(a - b)) < 1e-10


RANGES = r'''
import json, sys
import numpy as np
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.models.circuits import Circuit
from quest_amd.ops import capi
env = qa.Env()
n = int(sys.argv[2])
seeds = [int(x) for x in sys.argv[3].split(",")]
rows, states = [], []
for sd in seeds:
    r = qa.Register(env, n)
    r.init_plus()
    capi.resetQuESTStats()
    if sd < 0:
        # crafted: layers on the low qubits, then the top (rank) qubit joins --
        # its swap's first post-swap passes leave the high local positions
        # out of their tiles, so they run range by range
        rng = np.random.default_rng(-sd)
        lo = n - 6
        for layer in range(4):
            for q in range(lo):
                r.ry(q, float(rng.uniform(0, 3)))
            for q in range(layer % 2, lo - 1, 2):
                r.cnot(q, q + 1)
        r.h(n - 1)
        for layer in range(3):
            for q in list(range(0, lo, 2)) + [n - 1]:
                r.rx(q, float(rng.uniform(0, 3)))
            r.cnot(n - 1, 0)
    else:
        random_layered(n, 20, seed=sd).apply(r)
    r.sync()
    st = capi.getQuESTStats()
    rows.append({k: st[k] for k in ("swaps", "overlappedSwaps", "overlappedPasses")})
    states.append(r.to_numpy())
    r.close()
if env.rank == 0:
    np.save(sys.argv[1], np.array(states))
    print("STATS " + json.dumps(rows))
'''


@pytest.mark.parametrize("ranks", [2, 4])
def test_swap_ranges_overlap_random_circuits_rccl_shared_gpu(genv, tmp_path, ranks):
    """Receive-side swap overlap (round 6, be::swapRanges): RCCL ranks
    sharing the GPU, exchange slices small enough that every swap has 8
    ranges (QUEST_EXCHANGE_SLICE_KB).  A pass after a swap whose tile holds
    the incoming qubit cannot wait on one part; when it leaves the high local
    positions (the ranges' bits) out, it runs range by range as the ranges
    land -- and the passes after it that do too run with it range-major (each
    on range v as soon as v landed).  The first pass after such a swap keeps those positions out of its
    tile (router: q.firstPassAvoid -- their ops wait for the next pass), so
    every window, the crafted ones (-1, -2) and two bench seeds' 20-layer
    random layered ones, overlaps at least one pass per swap; the states
    equal the single-rank run's."""
    from quest_amd.parallel import spawn_local

    here = os.path.dirname(os.path.abspath(__file__))
    n = 22 + {2: 1, 4: 2}[ranks]
    # (all five bench seeds: profiles/r6/swap_ranges.txt; FUZZ-style override RANGES_SEEDS)
    seeds = os.environ.get("RANGES_SEEDS", "-1,-2,7,13" if ranks == 2 else "-1,-2,7")
    one, dist = str(tmp_path / "one.npy"), str(tmp_path / "dist.npy")
    base = {"QUEST_BACKEND": "hip", "PYTHONPATH": os.path.dirname(here)}
    import subprocess
    import sys

    p = subprocess.run([sys.executable, "-c", RANGES, one, str(n), seeds], env=dict(os.environ, **base),
                       capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    res = spawn_local(["-c", RANGES, dist, str(n), seeds], ranks,
                      env_extra=dict(base, QUEST_COMM="rccl", QUEST_RCCL_SHARED_GPU="1", QUEST_COMM_TIMEOUT="150",
                                     QUEST_EXCHANGE_SLICE_KB="512"), timeout=280)
    for r, q in enumerate(res):
        assert q.returncode == 0, f"rank {r}:\n{q.stdout[-1500:]}\n{q.stderr[-2500:]}"
    rows = json.loads([ln for ln in res[0].stdout.splitlines() if ln.startswith("STATS")][0][6:])
    print("per window (crafted x2, bench seeds):", rows)
    for row in rows:
        assert row["swaps"] >= 1 and row["overlappedSwaps"] >= 1, rows
    for row in rows:
        assert row["overlappedPasses"] >= row["overlappedSwaps"], rows
    # the bench seeds' windows: the first passes after the swap run as a
    # range-major chain (QUEST_SWAP_RANGES_FIRST: 3 for swaps of 1-2 qubits)
    for sd, row in zip(seeds.split(","), rows):
        if int(sd) >= 0:
            assert row["overlappedPasses"] >= 3 * row["overlappedSwaps"], rows
    a, b = np.load(one), np.load(dist)
    assert np.max(np.abs(a - b)) < 1e-10


def test_fork_benchmark_30q_matches_host_build(genv, tmp_path):
    """The fork's 30-qubit benchmark program (examples/random_circuit_benchmark.c
    flow: 490 gates, then P(q_i=1) for all 30 qubits and 10 amplitudes) on the
    GPU; the outputs must equal, to the printed digits, those of the host
    (CPU, OpenMP) build recorded in tests/data/fork_circuit_*_cpu.dat."""
    import quest_amd as qa
    from quest_amd.models import fork_circuit

    here = os.path.dirname(os.path.abspath(__file__))
    r = qa.Register(genv, 30)
    r.init_zero()
    qa.capi.resetQuESTStats()
    fork_circuit().apply(r)
    r.sync()
    st = qa.capi.getQuESTStats()
    assert st["wavePasses"] > 0 and st["wavePasses"] >= st["passes"] // 2, st  # the default engine ran it
    probs = [r.prob(i, 1) for i in range(30)]
    amps = [r.amp(i) for i in range(10)]
    want_p = [float(l.split(":")[1]) for l in open(os.path.join(here, "data", "fork_circuit_probs_cpu.dat"))
              if l.startswith("Probability")]
    want_a = [complex(*map(float, l.split(":")[1].split(","))) for l in
              open(os.path.join(here, "data", "fork_circuit_amps_cpu.dat"))]
    assert len(want_p) == 30 and len(want_a) == 10
    np.testing.assert_allclose(probs, want_p, atol=1.5e-6)
    np.testing.assert_allclose(np.array(amps), np.array(want_a), atol=1.5e-6)
    assert abs(r.total_prob() - 1) < 1e-10
    r.close()


@pytest.mark.parametrize("layout", [0, 1, 2])
@pytest.mark.parametrize("low_to_tile", [0, 1])
def test_direct_kernel_variants(genv, layout, low_to_tile):
    """Unfused gates through every direct-kernel variant (unit order, low
    targets in-register vs via the tile pass), 16 qubits, vs the oracle."""
    import quest_amd as qa
    from helpers import apply_random_ops, assert_close, oracle_for

    qa.capi.setGateFusion(0)
    qa.capi.setQuESTTuning("direct_layout", layout)
    qa.capi.setQuESTTuning("direct_low_to_tile", low_to_tile)
    rng = np.random.default_rng(10 * layout + low_to_tile)
    reg = qa.Register(genv, 16)
    o = oracle_for(reg, rng)
    apply_random_ops(reg, o, rng, 120)
    for t in range(16):  # every target, incl. the in-vector ones
        apply_random_ops(reg, o, rng, 0)
        reg.h(t)
        o.apply(np.array([[1, 1], [1, -1]]) / np.sqrt(2), t)
        reg.t(t)
        o.apply(np.diag([1, np.exp(1j * np.pi / 4)]), t)
    assert_close(reg, o)
    reg.close()


def test_direct_kernel_variants_fp32():
    """The fp32 unfused kernels (in-vector targets 0-1, lane-shuffle targets
    2-4, pair kernel above the line) under both launch layouts, 16 qubits, vs
    the oracle -- subprocess bound to the fp32 HIP library."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path.insert(0, 'tests')\n"
        "import numpy as np, quest_amd as qa\n"
        "from helpers import apply_random_ops, oracle_for, state_of\n"
        "from quest_amd.ops import capi\n"
        "assert capi.getQuEST_PREC() == 1\n"
        "e = qa.Env(); capi.setGateFusion(0)\n"
        "for lay in (1, 2):\n"
        "    for low in (0, 1):\n"
        "        capi.setQuESTTuning('direct_layout', lay); capi.setQuESTTuning('direct_low_to_tile', low)\n"
        "        rng = np.random.default_rng(lay * 10 + low)\n"
        "        r = qa.Register(e, 16); o = oracle_for(r, rng)\n"
        "        apply_random_ops(r, o, rng, 80)\n"
        "        for t in range(16):\n"
        "            r.h(t); o.apply(np.array([[1, 1], [1, -1]]) / np.sqrt(2), t)\n"
        "            r.t(t); o.apply(np.diag([1, np.exp(1j * np.pi / 4)]), t)\n"
        "        err = np.max(np.abs(state_of(r) - o.v)); r.close()\n"
        "        assert err < 2e-5, (lay, low, err)\n"
        "print('fp32 direct ok')\n"
    )
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, QUEST_BACKEND="hip", QUEST_PREC="1"))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "fp32 direct ok" in out.stdout


def test_tile_qubits_12_matches_oracle(genv):
    """The optional 64 KiB tile (tile_qubits = 12) on a long fused circuit."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.utils import oracle as O

    qa.capi.setQuESTTuning("tile_qubits", 12)
    qa.capi.setQuESTTuning("tile_mode", 0)
    n = 20
    c = random_layered(n, 8, seed=12)
    reg = qa.Register(genv, n)
    reg.init_plus()
    c.apply(reg)
    o = O.StateVector(n, np.full(1 << n, 1 / math.sqrt(1 << n)))
    c.apply_oracle(o)
    assert np.max(np.abs(reg.to_numpy() - o.v)) < 1e-10
    reg.close()


def test_reference_golden_suite_fp32_on_gpu():
    """The fp32 HIP library on the golden data (subprocess: one precision per
    process)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-m", "quest_amd.utils.golden", "--tol", "2e-4"], cwd=root,
                         env=dict(os.environ, QUEST_BACKEND="hip", QUEST_PREC="1"), capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "773 passed, 0 failed" in out.stdout


def test_checkpoint_round_trip_gpu(genv, tmp_path):
    """Binary checkpoint of a 24-qubit register (256 MiB) through host slices."""
    import quest_amd as qa
    from quest_amd.models import random_layered

    r = qa.Register(genv, 24)
    r.init_plus()
    random_layered(24, 2, seed=2).apply(r)
    want_p = [r.prob(q, 1) for q in (0, 11, 23)]
    amp = r.amp(12345)
    assert r.save(tmp_path / "ck")
    s = qa.Register(genv, 24)
    assert s.load(tmp_path / "ck")
    # the amplitudes come back bit for bit; the marginals only to rounding,
    # since the source register may sit in a relabelled qubit layout (its
    # sums run over the amplitudes in another order) and the loaded one in
    # the identity layout
    np.testing.assert_allclose([s.prob(q, 1) for q in (0, 11, 23)], want_p, rtol=0, atol=1e-14)
    assert s.amp(12345) == amp
    np.testing.assert_array_equal(s.to_numpy(), r.to_numpy())
    assert abs(s.inner(r) - 1) < 1e-12
    r.close()
    s.close()


def test_sync_watchdog_reports_unfinished_work():
    """QUEST_SYNC_TIMEOUT: a host wait on device work that takes longer than
    the limit ends the process with a report (the same polling wait carries
    the RCCL async-error / peer-timeout watchdog).  Subprocess: exits."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import quest_amd as qa\n"
            "from quest_amd.ops import capi\n"
            "env = qa.Env(); reg = qa.Register(env, 30)\n"
            "capi.setGateFusion(0)\n"
            "for _ in range(40):\n"
            "    reg.h(20)\n"
            "reg.sync()\n"
            "print('FINISHED')\n")
    envv = dict(os.environ, QUEST_BACKEND="hip", QUEST_SYNC_TIMEOUT="0.02")
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=envv, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode != 0 and "FINISHED" not in out.stdout, out.stdout
    assert "QUEST_SYNC_TIMEOUT" in out.stderr, out.stderr[-2000:]
    # and without the limit the same program completes
    envv.pop("QUEST_SYNC_TIMEOUT")
    ok = subprocess.run([sys.executable, "-c", code], cwd=root, env=envv, capture_output=True, text=True,
                        timeout=300)
    assert ok.returncode == 0 and "FINISHED" in ok.stdout, ok.stderr[-2000:]


@pytest.mark.parametrize("stream", ["1", "0"])
def test_relabelled_layout_reads_on_gpu(stream):
    """GPU twin of tests/test_relabel.py: a 22-qubit layered circuit on the
    wave engine with relabelling passes (streamed to the GPU pass by pass, or
    planned whole first: QUEST_PLAN_STREAM), then amplitudes, marginals,
    clones, inner products, setAmps and a checkpoint in the permuted layout,
    all against the NumPy oracle.  Subprocess: the knob is read once."""
    import subprocess
    import sys

    from test_relabel import ROOT, SCRIPT

    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, "22"], cwd=ROOT, capture_output=True, text=True,
                         timeout=240, env=dict(os.environ, QUEST_BACKEND="hip", QUEST_PLAN_STREAM=stream))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "relabel ok" in out.stdout
    moved = int(out.stdout.split("moved")[1].split()[0])
    assert moved > 0, out.stdout
