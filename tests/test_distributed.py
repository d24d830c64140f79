"""Distributed equivalence: the same workloads on 1
rank (in process) and on 2 / 4 ranks (one process per rank, CPU socket
transport, 127.0.0.1) must agree — state vectors, density matrices,
probabilities, seeded measurement outcomes, reductions and QASM text.  The
registers are small (6-12 qubits), so 1-2 of their qubits are global and
every gate kind crosses the rank boundary (global<->local swaps, control
bits on rank bits, chunk-level collapse)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)


def _free_port_pair():
    """A port P with P + 1 free as well: torchrun's store listens on P, the
    QuEST bootstrap on MASTER_PORT + 1 (src/comm/bootstrap.cpp) -- under
    parallel test workers another test's listener on P + 1 made the ranks
    greet the wrong process."""
    import socket

    for _ in range(64):
        a, b = socket.socket(), socket.socket()
        try:
            a.bind(("127.0.0.1", 0))
            port = a.getsockname()[1]
            b.bind(("127.0.0.1", port + 1))
            return port
        except OSError:
            continue
        finally:
            a.close()
            b.close()
    raise RuntimeError("no free port pair")


def _single(name, env):
    from scenarios import SCENARIOS

    return SCENARIOS[name](env)


def _multi(name, ranks, tmp_path, **env):
    from quest_amd.parallel import spawn_local

    out = str(tmp_path / f"{name}_{ranks}.npz")
    res = spawn_local([os.path.join(HERE, "dist_worker.py"), name, out], ranks,
                      env_extra={"QUEST_BACKEND": "cpu", "PYTHONPATH": ROOT, **env}, timeout=600)
    for r, p in enumerate(res):
        assert p.returncode == 0, f"rank {r}:\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}"
    with np.load(out, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("name", ["random_ops_statevector", "random_ops_density", "measurement_and_collapse",
                                  "calculations", "qasm_log", "top_swap"])
def test_distributed_equivalence(env, tmp_path, name, ranks):
    want = _single(name, env)
    got = _multi(name, ranks, tmp_path)
    assert int(got["_ranks"]) == ranks
    for k, v in want.items():
        g = got[k]
        if isinstance(v, str):
            assert str(g) == v, k
        else:
            np.testing.assert_allclose(np.asarray(g), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("ranks", [2, 4])
def test_rank_qubit_relabels(env, tmp_path, ranks):
    """X/Y/CNOT among rank qubits relabel chunks (no data moved) and diagonal
    gates on rank qubits scale per rank; reads, clone, inner products,
    checkpoints and measurement still see the logical state."""
    want = _single("rank_qubit_gates", env)
    got = _multi("rank_qubit_gates", ranks, tmp_path)
    for k, v in want.items():
        np.testing.assert_allclose(np.asarray(got[k]), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)
    assert int(got["_relabels"]) > 0
    assert int(got["_global_diags"]) > 0


@pytest.mark.parametrize("name", ["random_ops_statevector", "measurement_and_collapse", "rank_qubit_gates"])
def test_sliced_pipelined_exchange(env, tmp_path, name):
    """Tiny exchange slices (QUEST_EXCHANGE_SLICE_KB=1): every swap runs as
    many double-buffered slices (pack s+1 / exchange s / unpack s-1) and
    the canonical-placement restore in several pieces."""
    want = _single(name, env)
    got = _multi(name, 4, tmp_path, QUEST_EXCHANGE_SLICE_KB="1")
    for k, v in want.items():
        np.testing.assert_allclose(np.asarray(got[k]), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("ranks", [2, 4])
def test_wave_relabelling_with_rank_swaps(env, tmp_path, ranks):
    """Wave-planned ranks (host emulation, QUEST_CPU_PLANNER=3) whose passes
    relabel local qubits, under the router's rank-qubit swaps: the same state
    as one op-by-op process."""
    want = _single("layered_wave_relabel", env)
    got = _multi("layered_wave_relabel", ranks, tmp_path, QUEST_CPU_PLANNER="3")
    for k, v in want.items():
        if k.startswith("_"):
            continue
        np.testing.assert_allclose(np.asarray(got[k]), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)
    assert int(got["_swaps"]) > 0


def test_rank_controlled_ops_keep_layouts_aligned(env, tmp_path, monkeypatch):
    """24 qubits on 4 ranks (22 local, wave-planned by the host emulation): the
    bench's seed-13 circuit has CNOTs controlled by rank qubits.  Round 5 ran
    them only on the ranks whose bit is 1 (QUEST_RANK_TAGS=0), so the ranks'
    planners relabelled differently and every swap first had to bring the
    local layouts to rank 0's (router alignLayouts; without it the swaps cut
    their parts at different logical qubits: marginals off by 0.06 with the
    norm intact).  Round 6 queues them on every rank as rank-tagged ops
    (core.hpp kRankTagMask): the plans agree by construction and no rank ever
    aligns (tests/test_fuzz_dist.py: the plans themselves compared, and the
    control without tags diverging)."""
    import json

    monkeypatch.setenv("RCR_QUBITS", "24")
    want = _single("rank_controlled_relabel", env)
    got = _multi("rank_controlled_relabel", 4, tmp_path, QUEST_CPU_PLANNER="3", RCR_QUBITS="24")
    for k in ("probs", "amps", "norm"):
        np.testing.assert_allclose(np.asarray(got[k]), np.asarray(want[k]), rtol=0, atol=1e-11, err_msg=k)
    assert int(got["_swaps"]) > 0
    out = str(tmp_path / "rank_controlled_relabel_4.npz")
    aligns = [json.load(open(f"{out}.rank{r}.json"))["layoutAligns"] for r in range(4)]
    assert max(aligns) == 0, aligns


@pytest.mark.parametrize("name", ["random_ops_statevector", "calculations", "layered_wave_relabel"])
def test_eight_ranks(env, tmp_path, name):
    """The driver's 8-GPU shape (three rank qubits, all-to-all swaps among 8
    ranks, k = 3) rehearsed on the host transport."""
    want = _single(name, env)
    extra = {"QUEST_CPU_PLANNER": "3"} if name == "layered_wave_relabel" else {}
    got = _multi(name, 8, tmp_path, **extra)
    assert int(got["_ranks"]) == 8
    for k, v in want.items():
        if k.startswith("_"):
            continue
        g = got[k]
        if isinstance(v, str):
            assert str(g) == v, k
        else:
            np.testing.assert_allclose(np.asarray(g), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("ranks", [2, 8])
def test_restore_chunks_in_concurrent_rounds(env, tmp_path, ranks):
    """Chunk placement restored by concurrent rounds of pairwise whole-chunk
    exchanges (router restoreChunks): X on the rank qubits is one round that
    moves exactly one chunk per rank; CNOTs among rank qubits at most two."""
    want = _single("restore_chunks", env)
    got = _multi("restore_chunks", ranks, tmp_path)
    for k, v in want.items():
        if k.startswith("_"):
            continue
        np.testing.assert_allclose(np.asarray(got[k]), np.asarray(v), rtol=0, atol=1e-11, err_msg=k)
    chunk_bytes = 16 * (1 << (9 - {2: 1, 8: 3}[ranks]))
    assert int(got["_xor_rounds"]) == 1
    assert int(got["_xor_bytes"]) == chunk_bytes
    assert 1 <= int(got["_cyc_rounds"]) <= 2


def test_bench_under_torchrun_host_build():
    """bench.py in the driver's launch shape (torch.distributed.run, 4 ranks,
    127.0.0.1 rendezvous) on the host build: one JSON line from rank 0 with
    n_gpus 4, the state sharded over 4 ranks and qubit swaps performed."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port_pair()
    env = dict(os.environ, QUEST_BACKEND="cpu", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "QUEST_BOOTSTRAP_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "4", "--qubits", "14", "--steps", "3",
           "--warmup", "1", "--allow-transport"]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["config"]["qubits"] == 16
    assert d["config"]["swaps"] > 0 and d["config"]["norm_error"] < 1e-10


def test_swap_victims_survive_relabelling():
    """The bench window at 2 ranks x 28 qubits with the wave planner's
    relabelling passes (host emulation, plans only): ONE swap brings the rank
    qubit in.  Until round 3 the router chose the victim's physical position
    before flushing the backend, whose relabelling passes then put another
    qubit there: the swap moved a qubit the rest of the window still needed
    and a second full swap followed (2 instead of 1 per window at 2 ranks, 3
    instead of 1 at 8 ranks on the GPU)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port_pair()
    env = dict(os.environ, QUEST_BACKEND="cpu", QUEST_CPU_PLANNER="3", QUEST_PLAN_ONLY="1", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "QUEST_BOOTSTRAP_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--qubits", "28", "--steps", "20",
           "--warmup", "5", "--seed", "7", "--allow-transport", "--no-extras"]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert d["config"]["qubits"] == 29
    assert d["config"]["swaps"] == 1, d["config"]
