#!/usr/bin/env python3
"""Wall time of one window of the bench's layered circuit (30 qubits, 25
layers, seed 7: the per-pass overlap study's circuit) under the current
environment -- e.g. QUEST_WAVE_NOOPS=1 (loads / stores only) and planner
layout knobs -- best of --reps runs on fresh |+> states.

    QUEST_WAVE_NOOPS=1 QUEST_WAVE_LANE_ORDER=3 python tools/experiments/circuit_time.py
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--layers", type=int, default=25)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    env = qa.Env()
    reg = qa.Register(env, args.qubits)
    circ = random_layered(args.qubits, args.layers, seed=args.seed)
    ts = []
    for _ in range(args.reps):
        reg.init_plus()
        reg.sync()
        capi.resetQuESTStats()
        t0 = time.perf_counter()
        circ.apply(reg)
        reg.sync()
        ts.append(1e3 * (time.perf_counter() - t0))
    st = capi.getQuESTStats()
    knobs = {k: v for k, v in os.environ.items() if k.startswith("QUEST_WAVE") or k.startswith("QUEST_PLAN")}
    print(json.dumps({"ms": [round(t, 2) for t in ts], "best_ms": round(min(ts), 2), "passes": st["passes"],
                      "ms_per_pass": round(min(ts) / max(1, st["passes"]), 3), "knobs": knobs}), flush=True)


if __name__ == "__main__":
    main()
