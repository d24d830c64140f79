#!/usr/bin/env python3
"""Latency of one unfused gate + synchronisation at small sizes (launch /
sync bound): the metric's low-n end.  Run twice, with and without
QUEST_SYNC_TIMEOUT (which switches the wait from hipStreamSynchronize to a
polling loop), to compare the two waits.

    python tools/sync_latency.py [--qubits 16,20,22] [--reps 200]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", default="14,16,18,20,22")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    capi.setGateFusion(0)
    wait = "poll" if os.environ.get("QUEST_SYNC_TIMEOUT") else "hipStreamSynchronize"
    for n in [int(x) for x in args.qubits.split(",")]:
        r = qa.Register(env, n)
        r.init_plus()
        out = []
        for name, fn in (("h+sync", lambda: (r.h(n // 2), r.sync())), ("sync", r.sync),
                         ("h x10 + sync", lambda: ([r.h(n // 2) for _ in range(10)], r.sync()))):
            fn()
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            out.append(f"{name} {1e6 * ts[len(ts) // 2]:7.1f} us")
        print(f"n={n:2d} [{wait}] " + " | ".join(out), flush=True)
        r.close()


if __name__ == "__main__":
    main()
