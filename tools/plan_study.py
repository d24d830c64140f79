#!/usr/bin/env python3
"""Pass counts of the wave planner without touching the state (host build,
QUEST_PLAN_ONLY=1): the bench's layered circuit at full size in seconds.

    python tools/plan_study.py [--qubits 30] [--layers 25] [--warmup 5]
    (env knobs of the planner, e.g. QUEST_WAVE_RELABEL=0, QUEST_WAVE_CMIN=5)
"""
import argparse
import os
import sys

os.environ.setdefault("QUEST_BACKEND", "cpu")
os.environ.setdefault("QUEST_CPU_PLANNER", "3")
os.environ["QUEST_PLAN_ONLY"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--layers", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--window1", action="store_true", help="flush after every layer (bench.py window1_s_per_gate)")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit

    n = args.qubits
    env = qa.Env()
    reg = qa.Register(env, n)
    total = args.warmup + args.layers
    circ = random_layered(n, total, seed=args.seed)
    per, i = [], 0
    for layer in range(total):
        cnt = n + len(range(layer % 2, n - 1, 2))
        per.append(circ.gates[i:i + cnt])
        i += cnt
    for w in range(args.warmup):
        Circuit(n, per[w]).apply(reg)
    reg.flush()
    qa.capi.resetQuESTStats()
    for s in range(args.layers):
        Circuit(n, per[args.warmup + s]).apply(reg)
        if args.window1:
            reg.flush()
    reg.flush()
    st = qa.capi.getQuESTStats()
    print(f"qubits {n} layers {args.layers}: passes {st['passes']} wave {st['wavePasses']} "
          f"({st['passes'] / args.layers:.2f} per layer)")


if __name__ == "__main__":
    main()
