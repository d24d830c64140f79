#!/usr/bin/env python3
"""Does the register placement probe pick a fast re/im distance?  Creates
registers one after another (all kept alive, so each lands elsewhere) and
times the unfused Hadamard (direct streaming kernel) on three targets of each;
with QUEST_ALLOC_VERBOSE=1 the probe's table per register is on stderr.

    QUEST_ALLOC_VERBOSE=1 python tools/experiments/placement_check.py --qubits 30 --count 6
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--count", type=int, default=6)
    args = ap.parse_args()
    import quest_amd as qa

    env = qa.Env()
    n = args.qubits
    regs = []
    traffic = 4.0 * 8 * (1 << n)
    for k in range(args.count):
        r = qa.Register(env, n)
        r.init_plus()
        r.sync()
        regs.append(r)
        out = []
        for t in (0, n // 2, n - 1):
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                r.h(t)
                r.sync()
                ts.append(time.perf_counter() - t0)
            out.append(traffic / min(ts) / 1e12)
        print(f"register {k}: unfused H TB/s " + " ".join(f"t{t}={v:.2f}" for t, v in zip((0, n // 2, n - 1), out)),
              flush=True)


if __name__ == "__main__":
    main()
