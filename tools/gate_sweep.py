#!/usr/bin/env python3
"""Single-qubit-gate time vs #qubits (the BASELINE.json metric), per target
position, for eager (one pass per gate) and fused execution.

Prints one JSON line per measurement and a summary table; effective bandwidth
counts one read + one write of the whole fp64 state (2^(n+5) bytes) per pass.

    python tools/gate_sweep.py --min 20 --max 33 [--reps 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reg, reps):
    reg.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    reg.sync()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min", type=int, default=20)
    ap.add_argument("--max", type=int, default=30)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    rows = []
    for n in range(args.min, args.max + 1):
        reg = qa.Register(env, n)
        reg.init_plus()
        bytes_per_pass = (1 << n) * 32 if capi.binding().prec == 2 else (1 << n) * 16
        for target in sorted({0, 3, n // 2, n - 1}):
            capi.setGateFusion(0)
            reg.h(target)  # warm
            t_h = timed(lambda: reg.h(target), reg, args.reps)
            t_rx = timed(lambda: reg.rx(target, 0.3), reg, args.reps)
            t_t = timed(lambda: reg.t(target), reg, args.reps)
            c = (target + 1) % n
            t_cx = timed(lambda: reg.cnot(c, target), reg, args.reps)
            capi.setGateFusion(1)
            row = {"n": n, "target": target, "hadamard_s": t_h, "rotateX_s": t_rx, "tGate_s": t_t,
                   "controlledNot_s": t_cx, "GBps_hadamard": bytes_per_pass / t_h / 1e9}
            rows.append(row)
            print(json.dumps(row), flush=True)
        # fused: a layer of single-qubit gates on every qubit
        capi.setGateFusion(1)
        capi.resetQuESTStats()

        def layer():
            for q in range(n):
                reg.rx(q, 0.1 * (q + 1))

        t_layer = timed(layer, reg, max(2, args.reps // 4))
        st = capi.getQuESTStats()
        row = {"n": n, "fused_layer_s": t_layer, "fused_s_per_gate": t_layer / n,
               "passes_per_layer": st["passes"] / max(2, args.reps // 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        reg.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
