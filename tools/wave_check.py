#!/usr/bin/env python3
"""GPU check of the wave-tile engine (tile mode 3): random gate streams vs
the NumPy oracle at sizes where fused passes use 2^11-amplitude tiles, then
interleaved timing of tile modes 0 and 3 on the bench's layered circuit.

    python tools/wave_check.py [--qubits 30] [--layers 6] [--rounds 3]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="0,3")
    ap.add_argument("--skip-check", action="store_true")
    ap.add_argument("--wg", default="", help="comma list of wave_wg_per_cu values to time (mode 3)")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    env = qa.Env()
    if not args.skip_check:
        from helpers import apply_random_ops, oracle_for

        capi.setQuESTTuning("tile_mode", 3)
        for n in (20, 21, 23):
            rng = np.random.default_rng(n)
            reg = qa.Register(env, n)
            o = oracle_for(reg, rng)
            capi.resetQuESTStats()
            apply_random_ops(reg, o, rng, 600)
            err = float(np.max(np.abs(reg.to_numpy() - o.v)))
            st = capi.getQuESTStats()
            print(f"check n={n}: max err {err:.3e} passes {st['passes']} wave {st['wavePasses']}", flush=True)
            assert err < 1e-10, err
            assert st["wavePasses"] > 0
            reg.close()
        # mode 3 vs mode 0 on a layered circuit
        n = 24
        outs = {}
        for mode in (0, 3):
            capi.setQuESTTuning("tile_mode", mode)
            reg = qa.Register(env, n)
            reg.init_plus()
            random_layered(n, 8, seed=11).apply(reg)
            outs[mode] = reg.to_numpy()
            reg.close()
        d = float(np.max(np.abs(outs[0] - outs[3])))
        print(f"check layered n={n}: mode 3 vs 0 max diff {d:.3e}", flush=True)
        assert d < 1e-11

    n = args.qubits
    modes = [int(m) for m in args.modes.split(",")]
    variants = [(m, None) for m in modes]
    if args.wg:
        variants = [(3, int(w)) for w in args.wg.split(",")]
    reg = qa.Register(env, n)
    reg.init_plus()
    circ = random_layered(n, args.layers, seed=7)
    times = {v: [] for v in variants}
    stats = {}
    for r in range(args.rounds):
        for m in variants:
            capi.setQuESTTuning("tile_mode", m[0])
            if m[1] is not None:
                capi.setQuESTTuning("wave_wg_per_cu", m[1])
            reg.sync()
            capi.resetQuESTStats()
            t0 = time.perf_counter()
            circ.apply(reg)
            reg.sync()
            times[m].append(time.perf_counter() - t0)
            stats[m] = capi.getQuESTStats()
    g = len(circ.gates)
    for m in variants:
        best = min(times[m])
        print(f"mode {m[0]} wg {m[1]}: {1e3 * best / g:.4f} ms/gate ({1e3 * best / args.layers:.2f} ms/layer) "
              f"passes {stats[m]['passes']} wave {stats[m]['wavePasses']} all {[round(1e3 * t, 1) for t in times[m]]}",
              flush=True)
    print("norm", reg.total_prob())


if __name__ == "__main__":
    main()
