"""Deterministic workloads whose results must not depend on how many ranks
run them (distributed-equivalence tests).  Each
scenario takes an ``Env`` and returns a dict of numpy arrays / numbers,
identical on every rank."""
from __future__ import annotations

import numpy as np

from helpers import apply_random_noise, apply_random_ops


class NullOracle:
    """Stands in for the oracle in helpers.apply_* (only the register runs)."""

    def __getattr__(self, name):
        return lambda *a, **k: None


def random_ops_statevector(env):
    import quest_amd as qa

    rng = np.random.default_rng(7)
    r = qa.Register(env, 10)
    r.init_plus()
    apply_random_ops(r, NullOracle(), rng, 300)
    out = {"state": r.to_numpy(), "probs": np.array([r.prob(q, 1) for q in range(10)]),
           "norm": r.total_prob()}
    r.close()
    return out


def random_ops_density(env):
    import quest_amd as qa

    rng = np.random.default_rng(8)
    r = qa.Register(env, 5, density=True)
    r.init_plus()
    apply_random_ops(r, NullOracle(), rng, 80, noise=True)
    for _ in range(10):
        apply_random_noise(r, NullOracle(), rng)
    out = {"state": r.to_numpy(), "purity": r.purity(), "trace": r.total_prob(),
           "probs": np.array([r.prob(q, 0) for q in range(5)])}
    r.close()
    return out


def measurement_and_collapse(env):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    r = qa.Register(env, 12)
    r.init_plus()
    random_layered(12, 4, seed=3).apply(r)
    capi.seedQuEST([11, 22, 33], 3)
    outcomes = [r.measure(q) for q in (11, 0, 6, 3)]
    p = r.collapse(9, 1) if r.prob(9, 1) > 1e-6 else r.collapse(9, 0)
    ms = [r.measure_with_stats(q) for q in (1, 10)]
    out = {"outcomes": np.array(outcomes), "p": p, "ms": np.array(ms, dtype=float), "state": r.to_numpy()}
    d = qa.Register(env, 4, density=True)
    d.init_plus()
    d.h(3)
    d.cnot(3, 0)
    d.damping(0, 0.3)
    out["dens_outcomes"] = np.array([d.measure(q) for q in (0, 3, 2)])
    out["dens_state"] = d.to_numpy()
    r.close()
    d.close()
    return out


def calculations(env):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n = 9
    a, b = qa.Register(env, n), qa.Register(env, n)
    a.init_plus()
    random_layered(n, 3, seed=1).apply(a)
    b.init_classical(37)
    b.h(8)
    b.crx(8, 2, 0.7)
    out = {"inner": a.inner(b), "fid": a.fidelity(b), "amp": a.amp(300), "amp0": b.amp(37)}
    c = qa.Register(env, n)
    c.clone_from(a)
    c.ry(7, 0.4)
    out["clone_inner"] = c.inner(a)
    # density: initPureState, addDensityMatrix, fidelity vs pure, purity
    d1, d2 = qa.Register(env, 4, density=True), qa.Register(env, 4, density=True)
    p = qa.Register(env, 4)
    p.init_plus()
    p.rx(2, 1.1)
    p.cnot(2, 3)
    d1.init_pure(p)
    d2.init_classical(5)
    capi.addDensityMatrix(d1.q, 0.3, d2.q)
    out["dfid"] = d1.fidelity(p)
    out["dpur"] = d1.purity()
    out["dstate"] = d1.to_numpy()
    out["damp"] = d1.density_amp(5, 5)
    # setAmps across the rank boundary + getAmp
    e = qa.Register(env, 6)
    e.init_zero()
    vals = np.arange(20) * (0.01 + 0.02j)
    capi.setAmps(e.q, 22, vals.real, vals.imag, 20)
    out["setamps"] = e.to_numpy()
    capi.initStateOfSingleQubit(e.q, 4, 1)
    out["single"] = e.to_numpy()
    for r in (a, b, c, d1, d2, p, e):
        r.close()
    return out


def qasm_log(env):
    import quest_amd as qa

    r = qa.Register(env, 6)
    r.start_qasm()
    r.h(5)
    r.cnot(5, 0)
    r.crz(1, 4, 0.25)
    r.mcz([0, 2, 5])
    r.measure(5)
    text = r.qasm
    r.close()
    return {"qasm": text}


def rank_qubit_gates(env):
    """X/Y-like and diagonal gates on the top (rank) qubits, mixed with gates
    that do need a swap, then every read that depends on which rank holds
    which chunk: getAmp, probabilities, inner product with a register laid
    out differently, clone, measurement, a checkpoint round trip and the
    full state.  On >1 rank the anti-diagonal gates relabel chunks instead of
    moving data (the ``_relabels`` key, absent on one rank)."""
    import os
    import tempfile

    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n = 8
    r = qa.Register(env, n)
    r.init_plus()
    random_layered(n, 2, seed=5).apply(r)
    capi.canonicaliseQureg(r.q)   # logical qubits n-1.. on the rank bits
    capi.resetQuESTStats()
    for k in range(3):
        r.x(7)                # anti-diagonal on a rank qubit: relabel
        r.rz(7, 0.3 + k)      # diagonal on a rank qubit: per-rank scaling
        r.unitary(7, [[0, 0.6 + 0.8j], [1j, 0]])
        r.y(6)
        r.cnot(7, 6)
        r.t(6)
        r.z(7)
        r.s(6)
        r.phase(7, 0.2)
        r.x(6)
        r.cy(6, 7)            # rank control and target on 4 ranks
        r.h(2)
        r.cnot(1, 7)          # local control, rank target: needs data
        r.ry(5, 0.2)
    r.sync()
    st = capi.getQuESTStats()
    out = {"amps": np.array([r.amp(i) for i in (0, 5, 77, 200, 255)]),
           "probs": np.array([r.prob(q, 1) for q in range(n)])}
    b = qa.Register(env, n)
    b.init_plus()
    b.rx(7, 0.4)
    out["inner"] = r.inner(b)
    c = qa.Register(env, n)
    c.clone_from(r)
    c.x(7)
    c.h(0)
    out["clone_state"] = c.to_numpy()
    out["clone_inner"] = c.inner(r)
    r.x(6)
    # the ranks of one run are siblings: the parent's pid names a shared path
    path = os.path.join(tempfile.gettempdir(), f"qa_relabel_{env.num_ranks}_{os.getppid()}_{os.getpid() if env.num_ranks == 1 else 0}")
    assert r.save(path)
    r.x(7)
    assert r.load(path)
    out["state"] = r.to_numpy()
    capi.seedQuEST([5, 6], 2)
    r.x(7)
    out["outcomes"] = np.array([r.measure(q) for q in (7, 6, 0)])
    out["after"] = r.to_numpy()
    if env.num_ranks > 1:
        out["_relabels"] = st["relabels"]
        out["_global_diags"] = st["globalDiags"]
    for x in (r, b, c):
        x.close()
    return out


SCENARIOS = {f.__name__: f for f in (random_ops_statevector, random_ops_density, measurement_and_collapse,
                                     calculations, qasm_log, rank_qubit_gates)}


def checkpoint_save(env):
    """Build a state and write a checkpoint to $QA_CKPT (any rank count)."""
    import os

    import quest_amd as qa
    from quest_amd.models import random_layered

    r = qa.Register(env, 11)
    r.init_plus()
    random_layered(11, 3, seed=9).apply(r)
    assert r.save(os.environ["QA_CKPT"])
    out = {"state": r.to_numpy()}
    r.close()
    return out


def checkpoint_load(env):
    """Restore the checkpoint at $QA_CKPT (written by any rank count)."""
    import os

    import quest_amd as qa

    r = qa.Register(env, 11)
    assert r.load(os.environ["QA_CKPT"])
    out = {"state": r.to_numpy()}
    r.close()
    return out


SCENARIOS.update({f.__name__: f for f in (checkpoint_save, checkpoint_load)})


def layered_wave_relabel(env):
    """16 qubits, 14 layers: with QUEST_CPU_PLANNER=3 every rank runs wave
    passes that relabel its local qubits while the router swaps rank qubits
    in and out (the two layout mechanisms together)."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    r = qa.Register(env, 16)
    r.init_plus()
    random_layered(16, 14, seed=21).apply(r)
    probs = np.array([r.prob(q, 1) for q in range(16)])
    amps = np.array([r.amp(i) for i in (0, 1, 12345, 65535)])
    out = {"state": r.to_numpy(), "probs": probs, "amps": amps, "_swaps": capi.getQuESTStats()["swaps"]}
    r.close()
    return out


SCENARIOS["layered_wave_relabel"] = layered_wave_relabel


def rank_controlled_relabel(env):
    """21 qubits (19 local at 4 ranks: wave-sized, front flushes), the bench's
    layered circuit of seed 13: CNOTs controlled by rank qubits run only on the
    ranks whose bit is 1, so the ranks' planners see different op lists and
    relabel differently -- every swap must first bring the ranks' local
    layouts together (router alignLayouts)."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    import os

    from quest_amd.models.circuits import Circuit

    n = int(os.environ.get("RCR_QUBITS", "21"))
    r = qa.Register(env, n)
    r.init_plus()
    c = random_layered(n, 5, seed=13)
    per = len(c.gates) // 5 if hasattr(c, "gates") else None
    ops = list(c.gates) if per else None
    if ops:   # the bench's windows: one layer, then four (a sync after each)
        Circuit(n, ops[:per]).apply(r)
        r.sync()
        Circuit(n, ops[per:]).apply(r)
    else:
        c.apply(r)
    probs = np.array([r.prob(q, 1) for q in range(n)])
    amps = np.array([r.amp(i) for i in (0, 1, 777777, (1 << n) - 1)])
    st = capi.getQuESTStats()
    out = {"probs": probs, "amps": amps, "norm": r.total_prob(), "_swaps": st["swaps"], "_aligns": st["layoutAligns"]}
    r.close()
    return out


SCENARIOS["rank_controlled_relabel"] = rank_controlled_relabel


def hang_rank1(env):
    """Rank 1 stops responding; rank 0 must give up after QUEST_COMM_TIMEOUT."""
    import time

    import quest_amd as qa

    r = qa.Register(env, 8)
    r.init_plus()
    if env.rank == 1:
        time.sleep(120)
    p = r.total_prob()
    return {"p": p}


SCENARIOS["hang_rank1"] = hang_rank1


def restore_chunks(env):
    """X on every rank qubit relabels chunks (chunk c held by rank c ^ 7 on 8
    ranks); a read then restores the placement.  That permutation is an
    involution: ONE concurrent round of pairwise whole-chunk exchanges, one
    chunk per rank.  CNOTs among rank qubits make longer cycles: at most two
    rounds (a permutation is a product of two involutions)."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n = 9
    r = qa.Register(env, n)
    r.init_plus()
    random_layered(n, 2, seed=8).apply(r)
    capi.canonicaliseQureg(r.q)
    capi.resetQuESTStats()
    for q in (8, 7, 6):
        r.x(q)
    out = {"xor": r.to_numpy()}
    st = capi.getQuESTStats()
    out["_xor_rounds"], out["_xor_bytes"] = st["restoreRounds"], st["bytesExchanged"]
    capi.resetQuESTStats()
    r.x(8)
    r.cnot(8, 7)
    r.x(6)
    r.cnot(7, 6)
    r.cnot(6, 8)
    out["cycles"] = r.to_numpy()
    st = capi.getQuESTStats()
    out["_cyc_rounds"], out["_cyc_swaps"] = st["restoreRounds"], st["swaps"]
    r.close()
    return out


SCENARIOS["restore_chunks"] = restore_chunks


def top_swap(env):
    """Gates on qubits 0-5 and 7 of 8, qubit 6 idle: on 2 ranks the swap that
    brings rank qubit 7 in takes qubit 6, the top local position, so each
    part of the chunk is one contiguous range and RCCL sends it straight
    from the state (router multiSwap, no pack)."""
    import quest_amd as qa
    from quest_amd.ops import capi

    n = 8
    r = qa.Register(env, n)
    r.init_plus()
    rng = np.random.default_rng(9)
    capi.resetQuESTStats()
    for layer in range(3):
        for q in (0, 1, 2, 3, 4, 5, 7):
            r.ry(q, float(rng.uniform(0, 3)))
            r.rz(q, float(rng.uniform(0, 3)))
        for a in range(0, 5, 2):
            r.cnot(a, a + 1)
        r.cnot(5, 7)
    out = {"state": r.to_numpy(), "probs": np.array([r.prob(q, 1) for q in range(n)])}
    r.close()
    return out


SCENARIOS["top_swap"] = top_swap
