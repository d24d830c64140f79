#!/usr/bin/env python3
"""Cost of one fused tile pass as a function of the number of ops it holds.

Applies `m` gates on tile qubits 0..10 (so they land in ONE pass) and times
the pass for each tile mode; also times a torch device copy of the same
bytes as the streaming floor.

    python tools/experiments/pass_cost.py --qubits 30
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ops", default="1,2,4,8,16,32")
    ap.add_argument("--modes", default="0,2")
    ap.add_argument("--gates", default="h,t,cnot")
    args = ap.parse_args()

    import torch

    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    n = args.qubits
    reg = qa.Register(env, n)
    reg.init_plus()
    capi.setQuESTTuning("direct_kernels", 0)

    # streaming floor: read + write the two arrays once
    nbytes = (1 << n) * 8
    src = torch.empty(nbytes // 8, dtype=torch.float64, device="cuda")
    dst = torch.empty_like(src)
    ts = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src)
        dst.copy_(src)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    floor = statistics.median(ts)
    del src, dst
    torch.cuda.empty_cache()
    print(f"copy floor (2 arrays) {1e3 * floor:.3f} ms  {4 * nbytes / floor / 1e12:.2f} TB/s", flush=True)

    res = {"qubits": n, "copy_ms": 1e3 * floor, "runs": []}
    for mode in [int(x) for x in args.modes.split(",")]:
        capi.setQuESTTuning("tile_mode", mode)
        for g in args.gates.split(","):
            for m in [int(x) for x in args.ops.split(",")]:
                ts = []
                for _ in range(args.reps):
                    reg.sync()
                    capi.resetQuESTStats()
                    t0 = time.perf_counter()
                    for i in range(m):
                        q = i % 11
                        if g == "h":
                            reg.h(q)
                        elif g == "t":
                            reg.t(q)
                        else:
                            reg.cnot(q, (q + 1) % 11)
                    reg.sync()
                    ts.append(time.perf_counter() - t0)
                passes = capi.getQuESTStats()["passes"]
                t = statistics.median(ts)
                print(f"mode {mode} gate {g:4s} ops {m:3d}  passes {passes}  {1e3 * t:8.3f} ms/pass  "
                      f"{1e3 * (t - floor) / m:7.3f} ms/op over floor", flush=True)
                res["runs"].append({"mode": mode, "gate": g, "ops": m, "passes": passes, "ms": 1e3 * t})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
