#!/usr/bin/env python3
"""Per-gate-kind check of the wave-tile engine (tile mode 3) against the
NumPy oracle: streams of one gate type at a time on random qubits, so a
wrong handler shows up by name.  Also usable on the CPU build with
QUEST_CPU_PLANNER=3 (the host emulation of the same plans).

    python tools/wave_kinds.py [--qubits 18] [--count 24]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=18)
    ap.add_argument("--count", type=int, default=24)
    ap.add_argument("--kinds", default="")
    args = ap.parse_args()
    import quest_amd as qa
    from helpers import apply_named, oracle_for, GATES_1Q, GATES_2Q, GATES_MQ
    from quest_amd.ops import capi

    env = qa.Env()
    if capi.getQuESTBackend() == "HIP":
        capi.setQuESTTuning("tile_mode", 3)
    n = args.qubits
    kinds = args.kinds.split(",") if args.kinds else GATES_1Q + GATES_2Q + GATES_MQ
    bad = []
    for name in kinds:
        rng = np.random.default_rng(abs(hash(name)) % 1000)
        reg = qa.Register(env, n)
        o = oracle_for(reg, rng)
        capi.resetQuESTStats()
        for _ in range(args.count):
            k = 1 if name in GATES_1Q else 2 if name in GATES_2Q else int(rng.integers(2, 4))
            qs = [int(x) for x in rng.permutation(n)[:k]]
            apply_named(reg, o, name, qs, rng)
        err = float(np.max(np.abs(reg.to_numpy() - o.v)))
        st = capi.getQuESTStats()
        # amplitudes are ~2^(-n/2): fp32 keeps ~1e-7 of that per gate
        tol = 1e-10 if capi.binding().prec == 2 else 2e-6 * 2 ** (-n / 2) * args.count
        flag = "OK " if err < tol else "BAD"
        print(f"{flag} {name:10s} err {err:.3e} passes {st['passes']} wave {st['wavePasses']} "
              f"ops {st['waveOps']} tr {st['waveTransposes']}", flush=True)
        if err >= tol:
            bad.append(name)
        reg.close()
    print("bad:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
