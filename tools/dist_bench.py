#!/usr/bin/env python3
"""Distributed state-vector benchmark: R ranks x `qubits` local qubits, the
random layered circuit of bench.py, with the exchange accounting the
scaling analysis needs (swaps, bytes exchanged, time inside the all-to-all
qubit swaps, from the library's trace events).

One GPU (ranks share it through the device IPC transport, QUEST_COMM=ipc):

    python tools/dist_bench.py --ranks 4 --qubits 30          # spawns the ranks

Several GPUs (one rank per GPU over RCCL, started by torchrun):

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/dist_bench.py --worker --qubits 34

The 37-qubit / 8 x MI355X configuration of BASELINE.json is `--qubits 34` on 8
GPUs (256 GiB of state per GPU; getQuregMemoryPlan checks the budget first).
"""
import argparse
import json
import math
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(args):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit

    env = qa.Env()
    rank, world = env.rank, env.num_ranks
    n = args.qubits + int(round(math.log2(world)))
    plan = qa.capi.getQuregMemoryPlan(n, world)   # dict: state, exchange, scratch, total
    reg = qa.Register(env, n)
    reg.init_plus()
    layers = args.warmup + args.steps
    circ = random_layered(n, layers, seed=7)
    per = []
    i = 0
    for layer in range(layers):
        cnt = n + len(range(layer % 2, n - 1, 2))
        per.append(circ.gates[i:i + cnt])
        i += cnt
    for w in range(args.warmup):
        Circuit(n, per[w]).apply(reg)
    reg.sync()
    qa.capi.resetQuESTStats()
    env.sync()
    t0 = time.perf_counter()
    gates = 0
    for s in range(args.steps):
        Circuit(n, per[args.warmup + s]).apply(reg)
        gates += len(per[args.warmup + s])
    reg.sync()
    env.sync()
    dt = time.perf_counter() - t0
    st = qa.capi.getQuESTStats()
    norm = reg.total_prob()
    # latency of a distributed scalar read (local reduction + allreduce of
    # one fp64 through the transport) and of an amplitude read (owner read +
    # broadcast), the reference's MPI_Allreduce / MPI_Bcast call sites
    reps = 20
    env.sync()
    t1 = time.perf_counter()
    for _ in range(reps):
        reg.total_prob()
    scalar_ms = 1e3 * (time.perf_counter() - t1) / reps
    t1 = time.perf_counter()
    for i in range(reps):
        reg.amp((i * 7919) % (1 << n))
    amp_ms = 1e3 * (time.perf_counter() - t1) / reps
    # isolated swaps: a Hadamard on a qubit that sits on a rank position
    # (every rank idle before and after), less a Hadamard on a local qubit
    L = args.qubits
    iso, local_h = [], []
    for _ in range(3):
        lay = qa.capi.getQubitLayout(reg.q)
        qg = next(q for q in range(n) if lay[q] >= L)
        ql = next(q for q in range(n) if lay[q] < L)
        env.sync()
        t1 = time.perf_counter()
        reg.h(ql)
        reg.sync()
        env.sync()
        local_h.append(1e3 * (time.perf_counter() - t1))
        t1 = time.perf_counter()
        reg.h(qg)
        reg.sync()
        env.sync()
        iso.append(1e3 * (time.perf_counter() - t1))
    swap_ms, swap_lpos, swap_direct = [], [], []
    tr = os.environ.get("QUEST_TRACE")
    if tr and os.path.exists(tr):
        for line in open(tr):
            ev = json.loads(line)
            if ev.get("ev") == "swap":
                swap_ms.append(ev.get("host_ms", 0.0))
                swap_lpos.append([ev.get("lpos", []), ev.get("in_out", [])])
                swap_direct.append(ev.get("direct", 0))
    res = {"rank": rank, "ranks": world, "qubits": n, "local_qubits": args.qubits,
           "transport": qa.capi.getQuESTTransport(), "s_per_gate": dt / max(gates, 1), "seconds": dt,
           "gates": gates, "passes": st["passes"], "swaps": st["swaps"], "bytes_exchanged": st["bytesExchanged"],
           "relabels": st["relabels"], "swap_host_ms": swap_ms, "swap_victim_positions": swap_lpos,
           "swap_direct": swap_direct, "norm_error": abs(norm - 1),
           "total_prob_ms": scalar_ms, "get_amp_ms": amp_ms,
           "isolated_swap_plus_h_ms": [round(x, 3) for x in iso], "local_h_ms": [round(x, 3) for x in local_h],
           "memory_plan_bytes": plan}
    out = args.out or os.environ.get("QUEST_DIST_BENCH_OUT")
    if out:
        with open(f"{out}.rank{rank}.json", "w") as f:
            json.dump(res, f)
    if rank == 0:
        print(json.dumps(res), flush=True)
    reg.close()


def launch(args):
    with tempfile.TemporaryDirectory() as d:
        env = {"QUEST_COMM": args.comm, "QUEST_DIST_BENCH_OUT": os.path.join(d, "res")}
        # per-rank trace files for the swap timings
        procs = []
        script = [os.path.abspath(__file__), "--worker", "--qubits", str(args.qubits), "--steps", str(args.steps),
                  "--warmup", str(args.warmup)]
        import subprocess

        from quest_amd.parallel import _free_port
        port = _free_port()
        for r in range(args.ranks):
            e = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.ranks), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                     QUEST_BOOTSTRAP_ADDR="127.0.0.1", QUEST_BOOTSTRAP_PORT=str(port),
                     QUEST_TRACE=os.path.join(d, f"trace{r}.jsonl"), **env)
            procs.append(subprocess.Popen([sys.executable] + script, env=e, stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True))
        outs = [p.communicate(timeout=args.timeout) for p in procs]
        for r, (p, (so, se)) in enumerate(zip(procs, outs)):
            if p.returncode != 0:
                print(f"rank {r} failed ({p.returncode}):\n{se[-3000:]}", file=sys.stderr)
                sys.exit(1)
        ranks = [json.load(open(os.path.join(d, f"res.rank{r}.json"))) for r in range(args.ranks)]
    worst = max(ranks, key=lambda x: x["seconds"])
    summary = {"ranks": args.ranks, "qubits": worst["qubits"], "local_qubits": args.qubits,
               "transport": ranks[0]["transport"], "s_per_gate": worst["s_per_gate"], "passes": ranks[0]["passes"],
               "swaps": ranks[0]["swaps"], "bytes_exchanged_per_rank": ranks[0]["bytes_exchanged"],
               "swap_host_ms_rank0": ranks[0]["swap_host_ms"],
               "swap_victim_positions": ranks[0]["swap_victim_positions"], "swap_direct": ranks[0]["swap_direct"],
               "norm_error": ranks[0]["norm_error"],
               "total_prob_ms": ranks[0]["total_prob_ms"], "get_amp_ms": ranks[0]["get_amp_ms"],
               "isolated_swap_plus_h_ms": ranks[0]["isolated_swap_plus_h_ms"], "local_h_ms": ranks[0]["local_h_ms"],
               "memory_plan_bytes": ranks[0]["memory_plan_bytes"]}
    print(json.dumps(summary))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--qubits", type=int, default=30, help="local qubits per rank")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--comm", default="ipc", help="QUEST_COMM for the spawned ranks (one GPU: ipc)")
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    worker(args) if args.worker else launch(args)


if __name__ == "__main__":
    main()
