"""Seeded random programs for the distributed fuzz (tests/test_fuzz_dist.py).

    python tests/fuzz_dist.py <seed_lo> <seed_hi> <out_prefix>

Every rank runs programs seed_lo .. seed_hi - 1, one after another, in one
process; rank 0 writes ``<out_prefix>.npz`` (per seed: final state, reads
taken mid-circuit, measurement outcomes, reductions), every rank writes
``<out_prefix>.rank<r>.json`` with its own counters (layout alignments,
swaps, relabels).  The same command on 1 rank is the reference.

A program mixes what makes ranks diverge or move data: gates controlled by
qubits that sit on rank bits (the router's rank predicates), X / Y / phases
on rank qubits (chunk relabels, per-rank diagonals), seeded measurement and
collapse (chunk-level on rank qubits), reads in the middle (probabilities,
amplitudes, norms -- each flushes and may restore layouts), clones and inner
products of registers in different layouts, checkpoints saved and loaded,
and density registers under one- and two-qubit channels.
"""
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from helpers import GATES_1Q, GATES_2Q, apply_named  # noqa: E402


class _Null:
    def __getattr__(self, name):
        return lambda *a, **k: None


NULL = _Null()
SV_QUBITS = int(os.environ.get("FUZZ_SV_QUBITS", "16"))
DM_QUBITS = int(os.environ.get("FUZZ_DM_QUBITS", "6"))


def _gate(reg, rng, n, high):
    """One random gate; controls drawn from the top `high` qubits half the
    time (the qubits a swap-free program keeps on rank bits)."""
    kind = rng.random()
    if kind < 0.35:
        name = GATES_1Q[rng.integers(len(GATES_1Q))]
        t = int(rng.integers(n - high, n)) if rng.random() < 0.4 else int(rng.integers(n))
        apply_named(reg, NULL, name, [t], rng)
    elif kind < 0.8:
        name = GATES_2Q[rng.integers(len(GATES_2Q))]
        c = int(rng.integers(n - high, n)) if rng.random() < 0.5 else int(rng.integers(n))
        t = int(rng.integers(n))
        while t == c:
            t = int(rng.integers(n))
        apply_named(reg, NULL, name, [c, t], rng)
    else:
        k = int(rng.integers(2, 4))
        qs = list(rng.choice(n, size=k + 1, replace=False))
        name = ["mcunitary", "mcphase", "mcz"][rng.integers(3)]
        apply_named(reg, NULL, name, [int(x) for x in qs], rng)


def _noise(reg, rng, n):
    a, b = (int(x) for x in rng.choice(n, size=2, replace=False))
    k = int(rng.integers(5))
    p = float(rng.uniform(0, 0.4))
    [lambda: reg.dephase(a, p), lambda: reg.depolarise(a, p), lambda: reg.damping(a, p),
     lambda: reg.dephase2(a, b, p), lambda: reg.depolarise2(a, b, p)][k]()


def program(env, seed, tmpdir):
    import quest_amd as qa
    from quest_amd.ops import capi

    rng = np.random.default_rng(1000 + seed)
    out = {}
    n = SV_QUBITS
    a = qa.Register(env, n)
    a.init_plus()
    reads = []
    capi.seedQuEST([seed, 7], 2)
    outcomes = []
    nops = int(rng.integers(30, 90))
    for i in range(nops):
        _gate(a, rng, n, 3)
        r = rng.random()
        if r < 0.04:
            reads.append(a.prob(int(rng.integers(n)), 1))
        elif r < 0.07:
            z = a.amp(int(rng.integers(1 << n)))
            reads.extend([z.real, z.imag])
        elif r < 0.085:
            # (only qubits in superposition: a certain outcome's probability
            # is 1 +- 1e-13, and whether the draw is skipped at REAL_EPS --
            # the reference's rule -- depends on the summation order)
            q = int(rng.integers(n))
            if 1e-6 < a.prob(q, 0) < 1 - 1e-6:
                outcomes.append(a.measure(q))
        elif r < 0.095:
            # (the outcome is drawn, not thresholded on a probability: one
            # of exactly 0.5 rounds differently on different rank counts)
            q = int(rng.integers(n))
            o = int(rng.integers(2))
            if a.prob(q, o) < 1e-3:
                o = 1 - o
            reads.append(a.collapse(q, o))
    reads.append(a.total_prob())
    # a second register in another layout: clone, diverge, inner product
    b = qa.Register(env, n)
    b.clone_from(a)
    for _ in range(int(rng.integers(5, 20))):
        _gate(b, rng, n, 3)
    ip = a.inner(b)
    reads.extend([ip.real, ip.imag])
    # checkpoint round trip of b into a fresh register
    if rng.random() < 0.5:
        path = os.path.join(tmpdir, f"ck{seed}")
        assert b.save(path)
        c = qa.Register(env, n)
        assert c.load(path)
        for _ in range(5):
            _gate(c, rng, n, 3)
        out["ckpt_state"] = c.to_numpy()
        c.close()
    out["state"] = a.to_numpy()
    out["state_b"] = b.to_numpy()
    a.close()
    b.close()
    # density register with channels
    m = DM_QUBITS
    d = qa.Register(env, m, density=True)
    d.init_plus()
    for _ in range(int(rng.integers(10, 40))):
        if rng.random() < 0.6:
            _gate(d, rng, m, 2)
        else:
            _noise(d, rng, m)
        if rng.random() < 0.05:
            q = int(rng.integers(m))
            if 1e-6 < d.prob(q, 0) < 1 - 1e-6:
                outcomes.append(d.measure(q))
    reads.extend([d.purity(), d.total_prob()])
    out["dens"] = d.to_numpy()
    d.close()
    out["reads"] = np.array(reads, dtype=float)
    out["outcomes"] = np.array(outcomes, dtype=np.int64)
    return out


def main():
    import quest_amd as qa

    lo, hi, prefix = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    env = qa.Env()
    qa.capi.resetQuESTStats()
    res = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("FUZZ_TMP")) as tmp:
        # (ranks share the checkpoint directory: rank 0's, broadcast by name)
        shared = os.environ.get("FUZZ_CKPT_DIR", tmp)
        beat = os.environ.get("FUZZ_HEARTBEAT")   # (a progress line per program: long GPU runs)
        for seed in range(lo, hi):
            for k, v in program(env, seed, shared).items():
                res[f"{seed}/{k}"] = v
            if beat and env.rank == 0:
                with open(beat, "a") as f:
                    f.write(f"ranks {env.num_ranks} program {seed} done\n")
    st = qa.capi.getQuESTStats()
    with open(f"{prefix}.rank{env.rank}.json", "w") as f:
        json.dump({k: int(st[k]) for k in ("layoutAligns", "swaps", "relabels", "globalDiags", "passes",
                                          "wavePasses")}, f)
    if env.rank == 0:
        np.savez(f"{prefix}.npz", **res)
    env.close()


if __name__ == "__main__":
    main()
