#!/usr/bin/env python3
"""Bare streaming cost of a wave pass as a function of WHICH qubits form the
tile: one Hadamard on each of 13 chosen qubits makes a single pass whose
tile is exactly those qubits; run with QUEST_WAVE_NOOPS=1 the kernel only
loads and stores (no arithmetic), so the time is the memory system's
answer to that access pattern (2 x 16 B x 2^n bytes per pass).

    QUEST_WAVE_NOOPS=1 python tools/experiments/tile_layout_probe.py [--qubits 30]
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
    ap.add_argument("--only", default="", help="run only the sets whose name starts with this")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    reg = qa.Register(env, n)
    reg.init_plus()
    sets = {
        # tile sets of the round-4 bench passes (profiles/r4/overlap_study_r4b.txt; slowest and fastest)
        "r4 p0 0-7,9-13": [0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12, 13],
        "r4 p1 14,15,21-23,25": [0, 1, 2, 3, 4, 5, 6, 14, 15, 21, 22, 23, 25],
        "r4 p9 13,14,23-26": [0, 1, 2, 3, 4, 5, 6, 13, 14, 23, 24, 25, 26],
        "r4 p7 7,8,10,18-20": [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 18, 19, 20],
        "r4 p18 7,10,13,19,22,24": [0, 1, 2, 3, 4, 5, 6, 7, 10, 13, 19, 22, 24],
        "contiguous 0-12": list(range(13)),
        "unfused H 15 (direct)": [15],
        "0-3 + 4-12 (same)": list(range(13)),
        "0-3 + every 3rd": [0, 1, 2, 3, 7, 10, 13, 16, 19, 22, 25, 27, 29],
        "0-3 + top 9": [0, 1, 2, 3] + list(range(n - 9, n)),
        "0-3 + 10-18": [0, 1, 2, 3] + list(range(10, 19)),
        "0-3 + 4-6 + top 6": [0, 1, 2, 3, 4, 5, 6] + list(range(n - 6, n)),
        "0-6 + 18-23": list(range(7)) + list(range(18, 24)),
        "0-3 + 9-17": [0, 1, 2, 3] + list(range(9, 18)),
        "0-3 + 14-22": [0, 1, 2, 3] + list(range(14, 23)),
        "0-3 + 4-6 + 12-17": [0, 1, 2, 3, 4, 5, 6] + list(range(12, 18)),
    }
    traffic = 2 * 16 * (1 << n)
    for name, qs in sets.items():
        if args.only and not name.startswith(args.only):
            continue
        ts = []
        for _ in range(args.reps):
            reg.sync()
            capi.resetQuESTStats()
            t0 = time.perf_counter()
            for q in qs:
                reg.h(q)
            reg.sync()
            ts.append(time.perf_counter() - t0)
        st = capi.getQuESTStats()
        t = sorted(ts)[len(ts) // 2]
        print(f"{name:22s} {1e3 * t:8.3f} ms  {traffic / t / 1e12:5.2f} TB/s  passes {st['passes']} wave {st['wavePasses']}",
              flush=True)


if __name__ == "__main__":
    main()
