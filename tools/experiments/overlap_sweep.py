#!/usr/bin/env python3
"""How well the wave kernel overlaps arithmetic with the HBM stream: one
pass with k general one-qubit unitaries (+ CZs that stop them fusing) on
qubits inside one tile, for growing k.  A flat curve up to some k means the
ops hide under the stream; a line from k=0 means they add to it.

    python tools/experiments/overlap_sweep.py [--qubits 30]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ks", default="0,2,4,8,12,16,24,32,48")
    ap.add_argument("--kind", default="u", choices=["u", "h", "t", "x"])
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    capi.setQuESTTuning("tile_mode", 3)
    reg = qa.Register(env, args.qubits)
    reg.init_plus()
    u = [[0.6, 0.8j], [0.8j, 0.6]]
    qs = [0, 4, 5, 6]     # slot qubits of the first pass (tile bit 0 is slot 0)

    def gate(q):
        if args.kind == "u":
            reg.unitary(q, u)
        elif args.kind == "h":
            reg.h(q)
        elif args.kind == "t":
            reg.t(q)
        else:
            reg.x(q)

    def work(k):
        reg.t(1)
        reg.t(2)
        for i in range(k // 2):
            a, b = qs[(2 * i) % 4], qs[(2 * i + 1) % 4]
            gate(a)
            gate(b)
            reg.cz(a, b)

    base = None
    for k in [int(x) for x in args.ks.split(",")]:
        ts = []
        for _ in range(args.reps):
            reg.sync()
            capi.resetQuESTStats()
            t0 = time.perf_counter()
            work(k)
            reg.sync()
            ts.append(time.perf_counter() - t0)
        st = capi.getQuESTStats()
        t = min(ts)
        if base is None:
            base = t
        print(f"k={k:3d} ops {st['waveOps']:4d} passes {st['passes']} wave {st['wavePasses']}  "
              f"{1e3 * t:8.3f} ms  (+{1e3 * (t - base):7.3f} ms over k=0)", flush=True)


if __name__ == "__main__":
    main()
