#!/usr/bin/env python3
"""Placement / iteration-order probe for the unfused single-gate kernels:
H on target 0 and n/2 for several (allocation mode, im offset) placements of
the re/im arrays and both direct-kernel unit orders.

    python tools/experiments/layout_probe.py --qubits 28,29,30,31
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

PLACEMENTS = [("split", None), ("joint+0", 0), ("joint+4K", 4096), ("joint+1M4K", (1 << 20) + 4096),
              ("joint+2M", 2 << 20), ("joint+64M", 64 << 20)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", default="28,29,30,31")
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    capi.setGateFusion(0)
    for n in [int(x) for x in args.qubits.split(",")]:
        for label, off in PLACEMENTS:
            if off is None:
                os.environ["QUEST_ALLOC_MODE"] = "0"
            else:
                os.environ["QUEST_ALLOC_MODE"] = "1"
                os.environ["QUEST_IM_OFFSET"] = str(off)
            r = qa.Register(env, n)
            r.init_plus()
            row = []
            for lay in (0, 1):
                capi.setQuESTTuning("direct_layout", lay)
                for t in (0, n // 2):
                    ts = []
                    for _ in range(args.reps):
                        r.sync()
                        t0 = time.perf_counter()
                        r.h(t)
                        r.sync()
                        ts.append(time.perf_counter() - t0)
                    med = statistics.median(ts)
                    row.append(f"L{lay} t{t:<2d} {1e3 * med:8.3f} ms {32 * (1 << n) / med / 1e12:5.2f} TB/s")
            print(f"n={n} {label:11s} | " + " | ".join(row), flush=True)
            r.close()
    capi.setQuESTTuning("direct_layout", 0)


if __name__ == "__main__":
    main()
