#!/usr/bin/env python3
"""Per-op cost of the wave-tile kernel by gate kind: one pass of `count`
gates of a single kind on the low 10 qubits (all inside one tile) at
`qubits` qubits, timed against a pass of two phase gates (load + store +
dispatch only).  ms/op = (t_kind - t_base) / count.

    python tools/experiments/wave_micro.py [--qubits 28] [--count 32]
"""
import argparse
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=28)
    ap.add_argument("--count", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="regex: run only the matching workloads (plus the base pass)")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    capi.setQuESTTuning("tile_mode", 3)
    reg = qa.Register(env, args.qubits)
    reg.init_plus()
    c = args.count

    slot_q = [0, 4, 5, 6]          # tile bit 0 is slot 0; 4.. fill slots first
    lane_q = [1, 2, 3, 7, 8, 9]    # lanes 0-2 always; 3-5 the latest-used high bits
    workloads = {
        "base(2 phase)": lambda: (reg.t(0), reg.t(1)),
        "H slot (M2R)": lambda: [reg.h(slot_q[i % 4]) for i in range(c)],
        "Rx slot (M2RI)": lambda: [reg.rx(slot_q[i % 4], 0.3) for i in range(c)],
        "U slot (M2)": lambda: [reg.unitary(slot_q[i % 4], [[0.6, 0.8j], [0.8j, 0.6]]) for i in range(c)],
        "Y slot (ANTI)": lambda: [reg.y(slot_q[i % 4]) for i in range(c)],
        "X slot (SWAP)": lambda: [reg.x(slot_q[i % 4]) for i in range(c)],
        "T any (DIAG)": lambda: [reg.t(i % 10) for i in range(c)],
        "Rz slot (D2S)": lambda: [reg.rz(slot_q[i % 4], 0.3) for i in range(c)],
        "Rz lane (D2L)": lambda: [reg.rz(lane_q[i % 6], 0.3) for i in range(c)],
        "CNOT slot-slot": lambda: [reg.cnot(slot_q[i % 4], slot_q[(i + 1) % 4]) for i in range(c)],
        "CNOT lane->slot": lambda: [reg.cnot(lane_q[i % 6], slot_q[i % 4]) for i in range(c)],
        "H lanes 1-3 (TR l0-2)": lambda: [reg.h(1 + i % 3) for i in range(c)],
        "H lanes 7-9 (TR l3-5)": lambda: [reg.h(7 + i % 3) for i in range(c)],
        # 12 distinct qubits in one pass: some sit on wave bits (TRW through LDS)
        "H 12 qubits (TRW)": lambda: [(reg.h(i % 12), reg.cz(i % 12, (i + 1) % 12)) for i in range(c)],
        "H 10 qubits (no TRW)": lambda: [(reg.h(i % 10), reg.cz(i % 10, (i + 1) % 10)) for i in range(c)],
        # compute-bound: many ops in one pass (CZ breaks one-qubit fusion)
        "heavy M2 x200": lambda: [(reg.unitary(0, [[0.6, 0.8j], [0.8j, 0.6]]), reg.unitary(4, [[0.6, 0.8j], [0.8j, 0.6]]),
                                   reg.cz(0, 4)) for i in range(100)],
        "heavy M2R x200": lambda: [(reg.h(0), reg.h(4), reg.cz(0, 4)) for i in range(100)],
        "heavy DIAG x240": lambda: [reg.t(i % 4) for i in range(240)],
        "heavy TRl5 x120": lambda: [(reg.h(9), reg.h(8), reg.cz(8, 9)) for i in range(80)],
        # op lists that fit the scalar cache (~9 KB of records)
        "mid M2 x96": lambda: [(reg.unitary(0, [[0.6, 0.8j], [0.8j, 0.6]]), reg.unitary(4, [[0.6, 0.8j], [0.8j, 0.6]]),
                                reg.cz(0, 4)) for i in range(48)],
        "mid M2R x96": lambda: [(reg.h(0), reg.h(4), reg.cz(0, 4)) for i in range(48)],
        "mid DIAG x96": lambda: [reg.t(i % 4) for i in range(96)],
    }
    if args.only:
        import re

        workloads = {k: v for k, v in workloads.items() if k.startswith("base") or re.search(args.only, k)}
    res = {}
    for r in range(args.reps):
        for name, fn in workloads.items():
            reg.sync()
            capi.resetQuESTStats()
            t0 = time.perf_counter()
            fn()
            reg.sync()
            dt = time.perf_counter() - t0
            st = capi.getQuESTStats()
            res.setdefault(name, []).append((dt, st["wavePasses"], st["waveOps"], st["waveTransposes"], st["passes"]))
    base = min(x[0] for x in res["base(2 phase)"])
    hbm = 2 * 16 * (1 << args.qubits) / 6.3e12
    print(f"{args.qubits} qubits: one pass at 6.3 TB/s = {1e3 * hbm:.3f} ms; base pass {1e3 * base:.3f} ms")
    for name, v in res.items():
        dt = min(x[0] for x in v)
        _, wp, wo, tr, ps = v[0]
        per = (dt - base) / max(wo - 2, 1) if name != "base(2 phase)" else 0
        if name.startswith("heavy"):
            per = dt / max(wo, 1)
        print(f"{name:24s} {1e3 * dt:8.3f} ms  passes {ps} wave {wp} ops {wo} tr {tr}  "
              f"{1e6 * per:8.2f} us/op", flush=True)


if __name__ == "__main__":
    main()
