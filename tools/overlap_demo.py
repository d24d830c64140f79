#!/usr/bin/env python3
"""Overlapped qubit swaps on a workload that allows them (run under a 2-rank
launcher, e.g. tools/overlap_demo.sh): every window applies layers of
rotations and CNOTs to all local qubits except one (the victim of the coming
swap), then a Hadamard on the rank qubit and CNOTs from it into every other
qubit but the victim.  The router chooses that victim before the pre-swap
flush (it is outside the queued ops' targets), the passes of that flush leave
its position out of their tiles, and the backend runs them split around the
swap: the parts the swap sends first, the part it keeps next to the transfer
(QUEST_SWAP_OVERLAP).  The swapped-out victim is the next window's rank qubit.

Prints one JSON line: per-window wall times, swaps and split passes.

    python tools/overlap_demo.py --qubits 26 --windows 6 --layers 4
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=26, help="local qubits per rank")
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--layers", type=int, default=4, help="rotation + CNOT layers before each swap")
    args = ap.parse_args()
    import numpy as np
    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    ranks = env.num_ranks
    n = args.qubits + (ranks.bit_length() - 1)
    r = qa.Register(env, n)
    r.init_plus()
    r.sync()
    rng = np.random.default_rng(5)
    glob, victim = n - 1, args.qubits - 1     # the rank qubit the window needs, the local qubit it displaces
    times = []
    capi.resetQuESTStats()
    for w in range(args.windows):
        env.sync()
        t0 = time.perf_counter()
        busy = [q for q in range(n) if q not in (glob, victim)]
        for layer in range(args.layers):
            for q in busy:
                r.ry(q, float(rng.uniform(0, 3)))
            for i in range(layer % 2, len(busy) - 1, 2):
                r.cnot(busy[i], busy[i + 1])
        r.h(glob)
        for q in busy:
            r.cnot(glob, q)
        r.sync()
        times.append(time.perf_counter() - t0)
        # the victim left for the rank position: the next window's rank qubit
        glob, victim = victim, victim - 1 if victim > args.qubits - 8 else args.qubits - 1
        if victim == glob:
            victim -= 1
    st = capi.getQuESTStats()
    if env.rank == 0:
        print(json.dumps({"qubits": n, "ranks": ranks, "windows": args.windows, "layers": args.layers,
                          "window_ms": [round(1e3 * t, 3) for t in times],
                          "mean_ms_after_first": round(1e3 * sum(times[1:]) / max(1, len(times) - 1), 3),
                          "swaps": st["swaps"], "overlappedSwaps": st["overlappedSwaps"],
                          "overlappedPasses": st["overlappedPasses"], "swap_ms": st["swapMicros"] / 1e3,
                          "passes": st["passes"]}), flush=True)


if __name__ == "__main__":
    main()
