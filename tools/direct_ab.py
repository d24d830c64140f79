#!/usr/bin/env python3
"""Same-process A/B of the unfused (one gate = one pass) kernels: median wall
time of H on several targets and T on the middle qubit, for each setting of
the direct-kernel knobs (`direct_layout`, `direct_low_to_tile`), rounds
interleaved so slow drift of the box hits every setting alike.

    python tools/direct_ab.py [--qubits 30] [--reps 7] [--rounds 2]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    reg = qa.Register(env, n)
    reg.init_plus()
    capi.setGateFusion(0)
    traffic = 2 * 16 * (1 << n)
    settings = [(1, 1), (2, 1), (2, 0)]
    gates = [("h", 0), ("h", 1), ("h", 2), ("h", 3), ("h", 4), ("h", n // 2), ("h", n - 1), ("t", n // 2),
             ("t", 0)]
    best = {}
    for _ in range(args.rounds):
        for lay, low in settings:
            capi.setQuESTTuning("direct_layout", lay)
            capi.setQuESTTuning("direct_low_to_tile", low)
            for g, t in gates:
                fn = reg.h if g == "h" else reg.t
                fn(t)
                reg.sync()
                ts = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    fn(t)
                    reg.sync()
                    ts.append(time.perf_counter() - t0)
                m = sorted(ts)[len(ts) // 2]
                k = (lay, low, g, t)
                best[k] = min(best.get(k, 1e9), m)
    print(f"n={n}: median ms per unfused gate (best of {args.rounds} interleaved rounds), TB/s for H")
    print("gate  " + "".join(f"  layout={lay},low2tile={low}" for lay, low in settings))
    for g, t in gates:
        row = f"{g}({t:2d})"
        for lay, low in settings:
            m = best[(lay, low, g, t)]
            row += f"   {1e3 * m:7.3f} ms {traffic / m / 1e12 if g == 'h' else 0:4.2f}"
        print(row, flush=True)
    capi.setGateFusion(1)
    reg.close()


if __name__ == "__main__":
    main()
