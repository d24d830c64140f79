#!/usr/bin/env python3
"""Headline benchmark: single-qubit-gate time on a random fp64 state-vector
circuit (BASELINE.json: "single-qubit-gate time (s) vs #qubits, fp64
state-vector; 1/2/4/8-GPU scaling").

Workload (weak scaling): QUBITS_PER_GPU (default 30) qubits per GPU, so N
GPUs simulate 30 + log2(N) qubits, one rank per GPU (torchrun), the state
sharded over ranks and exchanged with RCCL over xGMI.  The workload is a
seeded random layered circuit: every layer is a random gate from {H, X, Y, Z,
S, T, Rx, Ry, Rz} on every qubit, then a brick layer of CNOTs (the fork
benchmark's gate mix, tutorial_example.c:29-518).  Five circuit seeds (7, and
11, 12, 13, 17, which no tuning ever used) run in one register each, every
one in its own window: K timed layers queued, then one sync, seed after seed.
A *step* is one layer of every seed's circuit.  `value` = wall seconds per
gate over all timed windows (the mean over the seeds; max over ranks), gates
applied through the public API exactly as a user would call them
(hadamard(), rotateX(), controlledNot(), ...).  `config.seeds` has each
seed's s/gate, window time and pass count (and at N > 1 its swaps, bytes sent
per rank, swap device time and the swap share of the window).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--qubits Q] [--seeds 7,11,...] [--eager] [--no-extras]

Besides the headline, a single-GPU run adds (outside the timed region, ~10 s):
  * ``sweep``: the metric's "vs #qubits" axis -- unfused Hadamard on targets
    0, n/2, n-1 and T on n/2 for n = 20, 22, ..., 32 (median of 5, one
    streaming pass per gate), with the achieved HBM bandwidth;
  * ``fork30``: the fork's own 30-qubit program end to end (490 gates, 30
    calcProbOfOutcome, 10 getAmp; tutorial_example.c:1-3, 29-534);
  * ``rotate29``: the reference's per-target benchmark
    (tests/benchmarks/rotate_benchmark.test): compactUnitary on every target
    of a 29-qubit register, 20 synced trials each, mean / stdev / min / max and
    TB/s per target;
  * ``window1_s_per_gate``: the seed-7 circuit flushed after every layer
    (the scheduler sees one layer at a time, as in a program that reads the
    state between layers);
  * ``fused_sweep``: the same axis on the fused path -- the five seeds'
    layered circuits (3 warm-up + 10 timed layers) at n = 20, 22, ..., 32 and
    34 (one seed, 20 layers): s/gate, passes and s/gate / 2^(n - 30);
  * ``q34``: 34 qubits (256 GiB, the largest state one MI355X holds): unfused
    H on targets 0 / 17 / 33 and a 6-layer random layered circuit;
  * ``density17``: a 17-qubit density matrix (2^34 amplitudes): damping,
    dephasing, two-qubit dephasing and depolarising per channel, gates;
  * ``fp32``: the headline circuit with the QUEST_PREC=1 library (a child
    process), its s/gate and the ratio to fp64.
  (--extras q34,fp32 picks some; --no-extras none; the extras use the first seed)
A multi-GPU run must use RCCL (``--allow-transport`` accepts another one).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_S_PER_OP = 3783.9266747315614 / 667  # fork's estimate, tutorial_example.c:1-3


DEFAULT_SEEDS = "7,11,12,13,17"   # 7: the rounds-1..4 headline; 11-13, 17 never used for tuning
FUSED_SWEEP_SEEDS = (7, 11, 12, 13, 17)


def split_layers(circ, n, layers):
    """The circuit's gates per layer (n one-qubit gates + a CNOT brick)."""
    out, i = [], 0
    for layer in range(layers):
        cnt = n + len(range(layer % 2, n - 1, 2))
        out.append(circ.gates[i:i + cnt])
        i += cnt
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20, help="timed layers of every seed's circuit")
    ap.add_argument("--warmup", type=int, default=5, help="untimed layers of every seed's circuit before")
    ap.add_argument("--qubits", type=int, default=30, help="qubits per GPU")
    ap.add_argument("--eager", action="store_true", help="disable gate fusion (one pass per gate)")
    ap.add_argument("--seeds", default=DEFAULT_SEEDS, help="comma-separated circuit seeds, one window each")
    ap.add_argument("--seed", type=int, default=None, help="a single circuit seed (overrides --seeds)")
    ap.add_argument("--no-extras", action="store_true", help="skip every extra (single-GPU runs only)")
    ap.add_argument("--extras", default="window1,fork30,sweep,rotate29,fused_sweep,q34,density17,fp32",
                    help="comma-separated extras of a single-GPU run")
    ap.add_argument("--allow-transport", action="store_true", help="accept a non-RCCL transport with N > 1")
    args = ap.parse_args()
    seeds = [args.seed] if args.seed is not None else [int(x) for x in args.seeds.split(",") if x]

    from quest_amd.parallel import allreduce_max, barrier, init_distributed, shutdown

    rank, world = init_distributed()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    import torch

    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())

    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit

    if args.eager:
        os.environ["QUEST_FUSION"] = "0"
    env = qa.Env()
    transport = qa.capi.getQuESTTransport()
    if world > 1 and not transport.startswith("RCCL") and not args.allow_transport:
        print(f"bench.py: {world} ranks must exchange over RCCL, transport is '{transport}'", file=sys.stderr)
        sys.exit(3)
    n = args.qubits + int(round(math.log2(world)))
    layers = args.warmup + args.steps
    # one register per seed (16 GiB each at 30 qubits per GPU), every one
    # warmed up with its own first W layers
    regs, per_seed_layers = [], []
    for sd in seeds:
        r = qa.Register(env, n)
        r.init_plus()
        lg = split_layers(random_layered(n, layers, seed=sd), n, layers)
        for w in range(args.warmup):
            Circuit(n, lg[w]).apply(r)
        r.sync()
        regs.append(r)
        per_seed_layers.append(lg)
    qa.capi.resetQuESTStats()

    # timed: every seed's K layers in its own window (queued, then one sync),
    # one seed after another; a step = one layer of every seed's circuit
    barrier()
    for r in regs:
        r.sync()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    gates = 0
    marks = []
    for r, lg in zip(regs, per_seed_layers):
        ts = time.perf_counter()
        g = 0
        for s in range(args.steps):
            Circuit(n, lg[args.warmup + s]).apply(r)
            g += len(lg[args.warmup + s])
        r.sync()
        st = qa.capi.getQuESTStats()
        marks.append((time.perf_counter() - ts, g, st["passes"], st["swaps"], st["bytesExchanged"],
                      st["swapMicros"], st["overlappedPasses"]))
        gates += g
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    barrier()
    elapsed = allreduce_max(time.perf_counter() - t0)
    stats = qa.capi.getQuESTStats()
    seed_rows, prev = [], (0, 0, 0, 0, 0)
    for sd, (dt, g, p, sw, by, us, ov) in zip(seeds, marks):
        dt = allreduce_max(dt)
        row = {"seed": sd, "s_per_gate": dt / max(g, 1), "window_ms": 1e3 * dt, "passes": p - prev[0]}
        if world > 1:
            swap_ms = allreduce_max((us - prev[3]) * 1e-3)
            row.update({"swaps": sw - prev[1], "swap_bytes_per_rank": by - prev[2], "swap_ms": swap_ms,
                        "swap_share": swap_ms / (1e3 * dt) if dt > 0 else None,
                        # wave passes launched while a swap was in flight (on the
                        # part it keeps, or range by range as ranges landed)
                        "overlapped_passes": int(allreduce_max(float(ov - prev[4])))})
        prev = (p, sw, by, us, ov)
        seed_rows.append(row)

    reg = regs[0]
    norm = reg.total_prob()  # sanity (outside the timed region)
    norm_err = max(abs(r.total_prob() - 1.0) for r in regs)
    for r in regs[1:]:
        r.close()
    # for reference, outside the timed region: one unfused gate (= one full
    # streaming pass over the state), median of 5
    qa.capi.setGateFusion(0)
    singles = []
    for _ in range(5):
        reg.sync()
        t1 = time.perf_counter()
        reg.h(n // 2)
        reg.sync()
        singles.append(time.perf_counter() - t1)
    qa.capi.setGateFusion(1)
    unfused_gate_s = allreduce_max(sorted(singles)[2])
    s_per_gate = elapsed / max(gates, 1)
    extras = {}
    if world == 1 and not args.no_extras and qa.capi.getQuESTBackend() == "HIP":
        try:
            extras = run_extras(qa, reg, n, per_seed_layers[0], args, seeds[0])   # closes reg
        except Exception as e:  # an optional extra must never cost the headline
            extras = {"extras_error": f"{type(e).__name__}: {e}"[:500]}
        if "s_per_gate" in extras.get("fp32", {}):
            extras["fp32"]["ratio_to_fp64"] = extras["fp32"]["s_per_gate"] / seed_rows[0]["s_per_gate"]
    else:
        reg.close()
    multi = {}
    if world > 1:
        swap_ms = sum(r["swap_ms"] for r in seed_rows)
        multi = {"swap_ms": swap_ms, "swap_bytes_per_rank": stats["bytesExchanged"],
                 "swap_share": swap_ms / (1e3 * elapsed) if elapsed > 0 else None,
                 "swap_GBps_per_rank": (stats["bytesExchanged"] / (swap_ms * 1e-3) / 1e9) if swap_ms > 0 else None,
                 # swaps before which some rank had to bring its local qubits to rank 0's positions
                 "layout_aligns_max": int(allreduce_max(float(stats["layoutAligns"]))),
                 "overlapped_swaps": stats["overlappedSwaps"], "overlapped_passes": stats["overlappedPasses"]}
    result = {
        "metric": "single-qubit-gate time (s) vs #qubits, fp64 state-vector; 1/2/4/8-GPU scaling",
        "value": s_per_gate,
        "unit": "s/gate",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / max(args.steps, 1),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": s_per_gate / BASELINE_S_PER_OP,
        "dtype": "fp64" if qa.capi.binding().prec == 2 else "fp32",
        "data": "synthetic: |+>^n initial state, seeded random layered circuits (one window per seed), random angles",
        "config": {
            "model": f"random layered circuits (1q gate on every qubit + CNOT brick), {n} qubits, "
                     f"seeds {','.join(map(str, seeds))}",
            "qubits": n,
            "qubits_per_gpu": args.qubits,
            "global_batch": len(seeds),
            "seq_len": 1 << n,
            "gates_per_step": gates / max(args.steps, 1),
            "parallelism": f"dp{world}: amplitude-sharded over {world} GPU(s)" +
                           ("" if world == 1 else ", all-to-all qubit swaps over " +
                            ("RCCL" if transport.startswith("RCCL") else transport)),
            "transport": transport,
            "fusion": not args.eager,
            "value_is": "mean s/gate over the seeds' windows (total time / total gates)",
            "seeds": seed_rows,
            "seed7_s_per_gate": next((r["s_per_gate"] for r in seed_rows if r["seed"] == 7), None),
            "passes": stats["passes"],
            "passes_per_seed": stats["passes"] / len(seeds),
            "swaps": stats["swaps"],
            **multi,
            "norm_error": max(abs(norm - 1.0), norm_err),
            "unfused_gate_s": unfused_gate_s,
            "backend": qa.capi.getQuESTBackend(),
            **extras,
        },
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    shutdown()


def _median_time(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def run_extras(qa, reg, n, layer_gates, args, seed):
    """Single-GPU extras, outside the timed region (see the module
    docstring); closes the bench register before the 256 GiB ones."""
    from quest_amd.models import fork_circuit
    from quest_amd.models.circuits import Circuit
    from quest_amd.utils.bench_workloads import run_density17, run_fused_sweep, run_q34, run_rotate29

    todo = set(args.extras.split(","))
    out = {}

    def guarded(key, fn):
        # each extra is optional: its failure is recorded, never raised
        try:
            fn()
        except Exception as e:
            out[key] = {"error": f"{type(e).__name__}: {e}"[:500]}

    def window1():
        # one-layer window: the same layers, flushed one at a time
        t0 = time.perf_counter()
        g = 0
        for s in range(args.steps):
            Circuit(n, layer_gates[args.warmup + s]).apply(reg)
            reg.flush()
            g += len(layer_gates[args.warmup + s])
        reg.sync()
        out["window1_s_per_gate"] = (time.perf_counter() - t0) / max(g, 1)

    def fork30():
        # fork program on a fresh register (the bench register stays allocated)
        fork = fork_circuit()
        f = qa.Register(reg.envobj, 30)
        f.init_zero()
        f.sync()
        t0 = time.perf_counter()
        fork.apply(f)
        f.sync()
        t1 = time.perf_counter()
        probs = [f.prob(q, 1) for q in range(30)]
        t2 = time.perf_counter()
        amps = [f.amp(i) for i in range(10)]
        t3 = time.perf_counter()
        out["fork30"] = {"total_s": t3 - t0, "gates_s": t1 - t0, "probs_s": t2 - t1, "amps_s": t3 - t2,
                         "gates": len(fork.gates), "p_q0": probs[0], "amp0": [amps[0].real, amps[0].imag]}
        f.close()

    def sweep_run():
        # unfused single-qubit gate time vs #qubits
        qa.capi.setGateFusion(0)
        sweep = []
        for m in range(20, 33, 2):
            r = qa.Register(reg.envobj, m)
            r.init_plus()
            r.sync()
            row = {"n": m}
            for name, t in (("h0", 0), ("hmid", m // 2), ("htop", m - 1), ("tmid", m // 2)):
                gate = r.h if name[0] == "h" else r.t

                def one():
                    gate(t)
                    r.sync()

                one()  # warm
                row[name + "_ms"] = 1e3 * _median_time(one)
            row["hmid_TBps"] = 2 * 16 * (1 << m) / (row["hmid_ms"] * 1e-3) / 1e12
            sweep.append(row)
            r.close()
        qa.capi.setGateFusion(1)
        out["sweep"] = sweep

    if "rotate29" in todo:
        res29 = {}
        guarded("rotate29", lambda: (run_rotate29(reg.envobj, res29), out.__setitem__("rotate29", res29["rotate29"])))
    if "window1" in todo:
        guarded("window1", window1)
    if "fork30" in todo:
        guarded("fork30", fork30)
    if "sweep" in todo:
        guarded("sweep", sweep_run)
        qa.capi.setGateFusion(1)
    env = reg.envobj
    reg.close()
    if qa.capi.binding().prec == 2:
        res = {}
        if "fused_sweep" in todo:
            guarded("fused_sweep", lambda: (run_fused_sweep(env, res, seeds=FUSED_SWEEP_SEEDS),
                                            out.__setitem__("fused_sweep", res["fused_sweep"])))
        if "q34" in todo:
            guarded("q34", lambda: (run_q34(env, res), out.__setitem__("q34", res["q34"])))
        if "density17" in todo:
            guarded("density17", lambda: (run_density17(env, res), out.__setitem__("density17", res["density17"])))
    if "fp32" in todo and qa.capi.binding().prec == 2:
        guarded("fp32", lambda: out.__setitem__("fp32", _run_fp32(args, seed)))
    return out


def _run_fp32(args, seed):
    """The headline circuit with the fp32 library, in a child process (a
    process binds one native library)."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--no-extras", "--steps", str(args.steps), "--warmup",
           str(args.warmup), "--qubits", str(args.qubits), "--seed", str(seed)]
    env = dict(os.environ, QUEST_PREC="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "fp32 child timed out after 300 s"}
    if p.returncode != 0:
        return {"error": p.stderr[-500:]}
    try:
        d = json.loads(p.stdout.strip().splitlines()[-1])
    except (IndexError, ValueError) as e:
        return {"error": f"fp32 child printed no JSON line: {e}"}
    return {"s_per_gate": d["value"], "passes": d["config"]["passes"], "norm_error": d["config"]["norm_error"],
            "unfused_gate_s": d["config"]["unfused_gate_s"], "dtype": d["dtype"]}


if __name__ == "__main__":
    main()
