#!/usr/bin/env python3
"""Streaming ceiling probe at `qubits` qubits (fp64): wall time of one pass
over the state by each engine with (almost) no arithmetic, next to a plain
device-to-device copy of the same bytes, all on the same box in one run.

    python tools/experiments/stream_probe.py [--qubits 30] [--reps 5]
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
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import quest_amd as qa
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    reg = qa.Register(env, n)
    reg.init_plus()
    traffic = 2 * 16 * (1 << n)

    def timeit(fn):
        ts = []
        for _ in range(args.reps):
            reg.sync()
            t0 = time.perf_counter()
            fn()
            reg.sync()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]

    def wave2():
        capi.setQuESTTuning("tile_mode", 3)
        reg.t(0)
        reg.t(1)

    def lds2():
        capi.setQuESTTuning("tile_mode", 0)
        reg.t(0)
        reg.t(1)

    def direct_h():
        capi.setGateFusion(0)
        reg.h(n // 2)
        capi.setGateFusion(1)

    res = {}
    for name, fn in (("wave pass (2 phase ops)", wave2), ("LDS tile pass (2 phase ops)", lds2),
                     ("direct H (unfused)", direct_h)):
        capi.resetQuESTStats()
        res[name] = (timeit(fn), capi.getQuESTStats()["passes"])
    capi.setQuESTTuning("tile_mode", 3)
    # plain copy of the same traffic: torch D2D copy of 16 B * 2^n
    a = torch.empty(1 << n, dtype=torch.complex128, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    ts = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.copy_(a)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res["torch copy_ (same bytes)"] = (sorted(ts)[len(ts) // 2], 0)
    for name, (t, p) in res.items():
        print(f"{name:30s} {1e3 * t:8.3f} ms  {traffic / t / 1e12:5.2f} TB/s  passes/{args.reps}: {p}", flush=True)


if __name__ == "__main__":
    main()
