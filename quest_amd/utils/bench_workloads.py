"""Benchmark workloads of every BASELINE.json configuration (shared by
bench.py's extras and tools/bench_suite.py).  Each ``run_*`` function adds
its results to the dict ``res``; all of them run through the public API
(quest_amd.Register) with the host blocking only where a program would.

  tutorial    3-qubit tutorial circuit (plumbing; P(|111>), P(q2=1))
  sweep       single-qubit-gate time vs #qubits, unfused (one pass per gate)
  random30    30-qubit fp64 depth-30 random layered circuit (fused)
  fork30      the fork's exact 30-qubit program (tutorial_example.c)
  q34         34 qubits (256 GiB state, one MI355X)
  qft30       30-qubit quantum Fourier transform on |+>^n
  density17   17-qubit density matrix (2^34 amplitudes) + noise channels
"""
import statistics
import time

FORK_ESTIMATE_S = 3783.9266747315614


def timed(fn, reps=5, sync=None):
    ts = []
    for _ in range(reps):
        if sync:
            sync()
        t0 = time.perf_counter()
        fn()
        if sync:
            sync()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), min(ts)


def run_tutorial(env, res):
    import quest_amd as qa

    q = qa.Register(env, 3)  # examples/tutorial_example.c
    q.init_zero()
    q.h(0)
    q.cnot(0, 1)
    q.ry(2, 0.1)
    q.mcz([0, 1, 2])
    u = [[0.5 + 0.5j, 0.5 - 0.5j], [0.5 - 0.5j, 0.5 + 0.5j]]
    q.unitary(0, u)
    q.compact(1, 0.5 + 0.5j, 0.5 - 0.5j)
    q.rotate(2, 3.14 / 2, (1, 0, 0))
    q.ccompact(0, 1, 0.5 + 0.5j, 0.5 - 0.5j)
    q.mcunitary([0, 1], 2, u)
    res["tutorial"] = {"prob_111": abs(q.amp(7)) ** 2, "prob_q2_1": q.prob(2, 1),
                       "reference": {"prob_111": 0.498751, "prob_q2_1": 0.749178}}
    q.close()


def run_sweep(env, res, max_q):
    import quest_amd as qa
    from quest_amd.ops import capi

    capi.setGateFusion(0)
    out = []
    for n in range(20, max_q + 1, 2):
        r = qa.Register(env, n)
        r.init_plus()
        row = {"qubits": n, "bytes_per_gate": 2 * 16 * (1 << n)}
        for label, t in (("t0", 0), ("mid", n // 2), ("top", n - 1)):
            med, mn = timed(lambda: r.h(t), reps=7 if n < 32 else 3, sync=r.sync)
            row[f"h_{label}_s"] = med
        med, _ = timed(lambda: r.t(n // 2), reps=7 if n < 32 else 3, sync=r.sync)
        row["t_mid_s"] = med
        row["h_mid_TBps"] = row["bytes_per_gate"] / row["h_mid_s"] / 1e12
        out.append(row)
        print(f"sweep n={n}: H t=0 {row['h_t0_s']*1e3:.3f} ms, mid {row['h_mid_s']*1e3:.3f} ms "
              f"({row['h_mid_TBps']:.2f} TB/s), top {row['h_top_s']*1e3:.3f} ms, T {row['t_mid_s']*1e3:.3f} ms",
              flush=True)
        r.close()
    capi.setGateFusion(1)
    res["sweep"] = out


def run_random30(env, res):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n, depth = 30, 30
    c = random_layered(n, depth, seed=30)
    r = qa.Register(env, n)
    r.init_plus()
    r.sync()
    capi.resetQuESTStats()
    t0 = time.perf_counter()
    c.apply(r)
    r.sync()
    dt = time.perf_counter() - t0
    st = capi.getQuESTStats()
    res["random30"] = {"gates": len(c.gates), "seconds": dt, "s_per_gate": dt / len(c.gates),
                       "passes": st["passes"], "norm_error": abs(r.total_prob() - 1)}
    print(f"random30: {len(c.gates)} gates in {dt:.3f} s ({1e3 * dt / len(c.gates):.3f} ms/gate, "
          f"{st['passes']} passes)", flush=True)
    r.close()


def run_qft30(env, res, n=30):
    """Quantum Fourier transform (H + n(n-1)/2 controlled phases) on |+>^n:
    the result is |0...0> (amp(0) = 1), a check as well as a timing."""
    import quest_amd as qa
    from quest_amd.models import qft
    from quest_amd.ops import capi

    c = qft(n)
    r = qa.Register(env, n)
    r.init_plus()
    r.sync()
    capi.resetQuESTStats()
    t0 = time.perf_counter()
    c.apply(r)
    r.sync()
    dt = time.perf_counter() - t0
    st = capi.getQuESTStats()
    a0 = r.amp(0)
    res["qft30"] = {"gates": len(c.gates), "seconds": dt, "s_per_gate": dt / len(c.gates), "passes": st["passes"],
                    "amp0_error": abs(a0 - 1)}
    print(f"qft{n}: {len(c.gates)} gates in {dt:.3f} s ({1e3 * dt / len(c.gates):.3f} ms/gate, {st['passes']} passes), "
          f"|amp0 - 1| = {abs(a0 - 1):.2e}", flush=True)
    r.close()


def run_fork30(env, res):
    import quest_amd as qa
    from quest_amd.models import fork_circuit

    c = fork_circuit()
    t0 = time.perf_counter()
    r = qa.Register(env, 30)
    r.sync()
    t1 = time.perf_counter()
    c.apply(r)
    r.sync()
    t2 = time.perf_counter()
    probs = [r.prob(i, 1) for i in range(30)]
    t3 = time.perf_counter()
    amps = [r.amp(i) for i in range(10)]
    t4 = time.perf_counter()
    dt = t4 - t0
    res["fork30"] = {"seconds": dt, "estimate_s": FORK_ESTIMATE_S, "speedup": FORK_ESTIMATE_S / dt,
                     "gates": len(c.gates), "create_s": t1 - t0, "gates_s": t2 - t1, "probs_s": t3 - t2,
                     "amps_s": t4 - t3, "prob_q0": probs[0], "amp0": [amps[0].real, amps[0].imag]}
    print(f"fork30: {dt:.3f} s (fork estimate {FORK_ESTIMATE_S:.1f} s, x{FORK_ESTIMATE_S / dt:.0f})", flush=True)
    r.close()


# the reference's per-target benchmark (tests/benchmarks/rotate_benchmark.test:8-57):
# compactUnitary with the first angle triple on every target of a 29-qubit
# |0...0> register, 20 trials per target
ROTATE_ANGLES = (1.2320, 0.4230, -0.6523)


def run_rotate29(env, res, n=29, trials=20):
    """compactUnitary on every target, each trial synced (the reference's CPU
    library returns when the gate is done; a GPU call returns at launch), with
    mean / stdev / min / max per target and the achieved HBM rate against the
    2^(n+5)-byte streaming floor of one read + one write of the state."""
    import math

    import quest_amd as qa

    a = ROTATE_ANGLES
    alpha = complex(math.cos(a[0]) * math.cos(a[1]), math.cos(a[0]) * math.sin(a[1]))
    beta = complex(math.sin(a[0]) * math.cos(a[2]), math.sin(a[0]) * math.sin(a[2]))
    q = qa.Register(env, n)
    q.init_zero()
    q.sync()
    nbytes = 2 * 16 * (1 << n)
    rows = []
    for t in range(n):
        q.compact(t, alpha, beta)   # warm this target's kernel
        q.sync()
        ts = []
        for _ in range(trials):
            t0 = time.perf_counter()
            q.compact(t, alpha, beta)
            q.sync()
            ts.append(time.perf_counter() - t0)
        mean = statistics.mean(ts)
        rows.append({"target": t, "mean_ms": 1e3 * mean, "stdev_ms": 1e3 * statistics.stdev(ts),
                     "min_ms": 1e3 * min(ts), "max_ms": 1e3 * max(ts), "TBps": nbytes / mean / 1e12})
    norm = q.total_prob()
    q.close()
    means = [r["mean_ms"] for r in rows]
    res["rotate29"] = {"qubits": n, "trials": trials, "bytes_per_gate": nbytes, "per_target": rows,
                       "mean_ms": statistics.mean(means), "slowest_ms": max(means), "fastest_ms": min(means),
                       "spread": max(means) / min(means), "norm_error": abs(norm - 1.0)}


def run_q34(env, res, n=34):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    r = qa.Register(env, n)
    r.init_plus()
    capi.setGateFusion(0)
    single = {}
    for label, t in (("t0", 0), ("mid", n // 2), ("top", n - 1)):
        single[label], _ = timed(lambda: r.h(t), reps=3, sync=r.sync)
    capi.setGateFusion(1)
    c = random_layered(n, 6, seed=34)   # 6 layers: the first layer alone is a poor average
    r.sync()
    t0 = time.perf_counter()
    c.apply(r)
    r.sync()
    dt = time.perf_counter() - t0
    res["q34"] = {"qubits": n, "state_GiB": 16 * (1 << n) / 2 ** 30, "h_single_s": single,
                  "layered_gates": len(c.gates), "layered_s_per_gate": dt / len(c.gates),
                  "norm_error": abs(r.total_prob() - 1)}
    print(f"q{n}: H {single}, layered {1e3 * dt / len(c.gates):.2f} ms/gate", flush=True)
    r.close()


def run_fused_sweep(env, res, seeds=(7, 11, 12, 13, 17), sizes=(20, 22, 24, 26, 28, 30, 32, 34), layers=10,
                    warmup=3, layers34=20):
    """The metric's "vs #qubits" axis on the fused path: the headline's
    seeded random layered circuits (one window of `layers` layers per seed
    after `warmup` untimed ones, |+>^n) at every size, one register per size
    re-initialised per seed.  Per size: s/gate (total time / total gates over
    the seeds), passes, and s/gate / 2^(n - 30) -- the per-amplitude rate
    against the 30-qubit one (1.0 = the same cost per byte).  34 qubits
    (256 GiB) runs `layers34` layers.  Below 23 qubits a wave pass has fewer
    tiles (2^(n - 13)) than the 768 resident workgroups of the chip, so
    small states pay occupancy and launch latency, not bandwidth."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit

    def split(circ, n, nl):
        out, i = [], 0
        for layer in range(nl):
            cnt = n + len(range(layer % 2, n - 1, 2))
            out.append(circ.gates[i:i + cnt])
            i += cnt
        return out

    rows = []
    for n in sizes:
        nl = layers34 if n >= 34 else layers
        r = qa.Register(env, n)
        tot_t, tot_g, tot_p = 0.0, 0, 0
        per_seed = []
        for sd in seeds:
            lg = split(random_layered(n, warmup + nl, seed=sd), n, warmup + nl)
            r.init_plus()
            for w in range(warmup):
                Circuit(n, lg[w]).apply(r)
            r.sync()
            p0 = qa.capi.getQuESTStats()["passes"]
            t0 = time.perf_counter()
            g = 0
            for w in range(warmup, warmup + nl):
                Circuit(n, lg[w]).apply(r)
                g += len(lg[w])
            r.sync()
            dt = time.perf_counter() - t0
            p = qa.capi.getQuESTStats()["passes"] - p0
            tot_t, tot_g, tot_p = tot_t + dt, tot_g + g, tot_p + p
            per_seed.append(round(dt / g, 9))
            if n >= 34:
                break   # one seed at 256 GiB (its window alone is ~1.5 s)
        spg = tot_t / tot_g
        rows.append({"n": n, "layers": nl, "seeds": len(per_seed), "s_per_gate": spg, "passes": tot_p,
                     "passes_per_layer": tot_p / (nl * len(per_seed)), "per_seed_s_per_gate": per_seed,
                     "scaled_to_30": spg / 2.0 ** (n - 30), "norm_error": abs(r.total_prob() - 1)})
        r.close()
    ref = next((x["scaled_to_30"] for x in rows if x["n"] == 30), None)
    for x in rows:
        x["per_byte_vs_30q"] = x["scaled_to_30"] / ref if ref else None
    res["fused_sweep"] = rows


def run_density17(env, res, n=17):
    import quest_amd as qa

    d = qa.Register(env, n, density=True)
    d.init_plus()
    d.sync()
    t0 = time.perf_counter()
    for q in range(n):
        d.damping(q, 0.1)
    d.sync()
    t_damp = (time.perf_counter() - t0) / n
    # dephasing (diagonal ops: they fuse into one pass) and two-qubit dephasing
    t0 = time.perf_counter()
    for q in range(n):
        d.dephase(q, 0.1)
    d.sync()
    t_deph = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for q in range(0, n - 1, 2):
        d.dephase2(q, q + 1, 0.1)
    d.sync()
    t_deph2 = (time.perf_counter() - t0) / len(range(0, n - 1, 2))
    t0 = time.perf_counter()
    for q in range(0, n - 1, 2):
        d.depolarise2(q, q + 1, 0.1)
    d.sync()
    t_dep2 = (time.perf_counter() - t0) / len(range(0, n - 1, 2))
    t0 = time.perf_counter()
    for q in range(n):
        d.depolarise(q, 0.1)
    d.sync()
    t_dep = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for q in range(n):
        d.h(q)
    for q in range(0, n - 1, 2):
        d.cnot(q, q + 1)
    d.sync()
    ng = n + len(range(0, n - 1, 2))
    t_gate = (time.perf_counter() - t0) / ng
    tr = d.total_prob()
    pur = d.purity()
    # a deeper random layered circuit (the q34 workload) on the density
    # matrix: each gate is U on the row qubit and conj(U) on the column qubit
    from quest_amd.models import random_layered

    c = random_layered(n, 6, seed=17)
    d.sync()
    t0 = time.perf_counter()
    c.apply(d)
    d.sync()
    t_layered = (time.perf_counter() - t0) / len(c.gates)
    res["density17"] = {"qubits": n, "amps": 1 << (2 * n), "damping_s_per_channel": t_damp,
                        "dephase_s_per_channel": t_deph, "dephase2_s_per_channel": t_deph2,
                        "depolarise_s_per_channel": t_dep, "depolarise2_s_per_channel": t_dep2,
                        "gate_s": t_gate, "layered_s_per_gate": t_layered, "trace": tr, "purity": pur}
    print(f"density{n}: damping {1e3 * t_damp:.2f} ms/channel, dephasing {1e3 * t_deph:.2f}, two-qubit "
          f"dephasing {1e3 * t_deph2:.2f} ms/channel, depolarising {1e3 * t_dep:.2f}, two-qubit depolarising "
          f"{1e3 * t_dep2:.2f} ms/channel, gates {1e3 * t_gate:.2f} ms/gate (one layer), "
          f"layered {1e3 * t_layered:.2f} ms/gate (6 layers), trace {tr:.12f}, purity {pur:.6f}", flush=True)
    d.close()
