#!/usr/bin/env python3
"""Workload for PMC counters of the unfused (direct) kernels: H on qubits 0
(in-vector kernel), 2 (lane-shuffle kernel) and n/2 (pair kernel), and T on
n/2 (diagonal kernel, half the state), 28 qubits, three of each.

    rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace -- python3 tools/experiments/direct_pmc.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import quest_amd as qa
    from quest_amd.ops import capi

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    env = qa.Env()
    r = qa.Register(env, n)
    r.init_plus()
    capi.setGateFusion(0)
    for fn, t in ((r.h, 0), (r.h, 2), (r.h, n // 2), (r.t, n // 2)):
        for _ in range(3):
            fn(t)
        r.sync()
    print("state bytes", 16 * (1 << n))
    r.close()


if __name__ == "__main__":
    main()
