#!/usr/bin/env python3
"""Same-process A/B of the pass scheduler's op cap (`plan_max_ops`) on the
headline workload: the 20 timed layers of bench.py's seeded random layered
circuit (30 qubits, one flush window), rounds interleaved across settings.

    python tools/plan_cap_ab.py [--qubits 30] [--rounds 3] [--caps 0,40,50,60,80]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--caps", default="0,40,50,60,80")
    ap.add_argument("--knob", default="plan_max_ops")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    reg = qa.Register(env, n)
    reg.init_plus()
    layers = args.warmup + args.steps
    circ = random_layered(n, layers, seed=7)
    chunks, i = [], 0
    for layer in range(layers):
        cnt = n + len(range(layer % 2, n - 1, 2))
        chunks.append(circ.gates[i:i + cnt])
        i += cnt
    timed = [g for c in chunks[args.warmup:] for g in c]
    Circuit(n, [g for c in chunks[:args.warmup] for g in c]).apply(reg)
    reg.sync()
    caps = [int(c) for c in args.caps.split(",")]
    res = {c: [] for c in caps}
    passes = {}
    for _ in range(args.rounds):
        for c in caps:
            capi.setQuESTTuning(args.knob, c)
            capi.resetQuESTStats()
            reg.sync()
            t0 = time.perf_counter()
            Circuit(n, timed).apply(reg)
            reg.sync()
            res[c].append((time.perf_counter() - t0) / len(timed))
            passes[c] = capi.getQuESTStats()["passes"]
    capi.setQuESTTuning(args.knob, caps[0])
    print(f"n={n}, {len(timed)} gates per run, {args.knob}: ms/gate (min, median over {args.rounds} rounds), passes")
    for c in caps:
        v = sorted(res[c])
        print(f"{args.knob}={c:4d}  {1e3 * v[0]:.4f}  {1e3 * v[len(v) // 2]:.4f}  passes {passes[c]}", flush=True)
    print(f"norm error {abs(reg.total_prob() - 1):.2e}")
    reg.close()


if __name__ == "__main__":
    main()
