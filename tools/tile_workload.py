#!/usr/bin/env python3
"""A fixed fused-pass workload for kernel profiling: `--ops` two-qubit
blocks (H, H, CNOT on a pair of tile qubits -> one 4x4 block each) per pass,
`--passes` passes, on `--qubits` qubits.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU ... -- python3 tools/tile_workload.py
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=28)
    ap.add_argument("--ops", type=int, default=16)
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--kind", default="mat4", choices=["mat4", "mat2", "diag"])
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    capi.setQuESTTuning("direct_kernels", 0)
    r = qa.Register(env, args.qubits)
    r.init_plus()
    r.sync()
    t0 = time.perf_counter()
    for _ in range(args.passes):
        for i in range(args.ops):
            a, b = i % 11, (i + 3) % 11
            if args.kind == "mat4":
                r.h(a)
                r.ry(b, 0.1 * i)
                r.cnot(a, b)
            elif args.kind == "mat2":
                r.h(a)
                r.t(a)  # forces no merge with the next H on another qubit only
            else:
                r.t(a)
        r.sync()
    dt = time.perf_counter() - t0
    st = capi.getQuESTStats()
    print(f"{args.kind}: {args.passes} passes x {args.ops}: {1e3 * dt / args.passes:.3f} ms/pass, stats {st}")


if __name__ == "__main__":
    main()
