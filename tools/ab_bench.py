#!/usr/bin/env python3
"""Interleaved A/B timing of backend variants in ONE process (rounds x
variants, median and min reported), for the random-layer workload of
bench.py.  Variants are (fusion, tuning-knob) settings applied at run time.

    python tools/ab_bench.py --qubits 28 --rounds 5
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = {
    "fused-noblocks": dict(fusion=1, tile_mode=0, direct_kernels=1, fuse_blocks=0),
    "fused-tile12": dict(fusion=1, tile_mode=0, direct_kernels=1, tile_qubits=12),
    "fused-dense": dict(fusion=1, tile_mode=2, direct_kernels=1),
    "fused-opbyop": dict(fusion=1, tile_mode=0, direct_kernels=1),
    "fused-regphase": dict(fusion=1, tile_mode=1, direct_kernels=1),
    "fused-wave": dict(fusion=1, tile_mode=3, direct_kernels=1),
    "eager-direct": dict(fusion=0, tile_mode=2, direct_kernels=1),
    "eager-tile": dict(fusion=0, tile_mode=2, direct_kernels=0),
}
# wave planner / kernel knobs (round 3: runtime tuning keys)
for _lo in (0, 1, 2):
    for _tm in (0, 1):
        VARIANTS[f"wave-lo{_lo}-tm{_tm}"] = dict(fusion=1, tile_mode=3, direct_kernels=1, wave_lane_order=_lo,
                                                 wave_tile_map=_tm)
DEFAULTS = {"tile_mode": 3, "direct_kernels": 1, "tile_wg_per_cu": 2, "fuse_blocks": 1, "tile_qubits": 0,
            "wave_lane_order": 1, "wave_tile_map": 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=28)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--circuit", default="layered", choices=["layered", "fork"])
    args = ap.parse_args()

    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    env = qa.Env()
    n = args.qubits
    reg = qa.Register(env, n)
    reg.init_plus()
    if args.circuit == "fork":
        from quest_amd.models import fork_circuit

        circ = fork_circuit() if n == 30 else __import__("quest_amd.models", fromlist=["x"]).fork_benchmark(n=n)
    else:
        circ = random_layered(n, args.layers, seed=5)
    names = args.variants.split(",")
    times = {v: [] for v in names}
    passes = {}
    for r in range(args.rounds):
        for v in names:
            cfg = VARIANTS[v]
            capi.setGateFusion(cfg["fusion"])
            for k, dv in DEFAULTS.items():
                capi.setQuESTTuning(k, cfg.get(k, dv))
            reg.sync()
            capi.resetQuESTStats()
            t0 = time.perf_counter()
            circ.apply(reg)
            reg.sync()
            times[v].append((time.perf_counter() - t0) / len(circ.gates))
            passes[v] = capi.getQuESTStats()["passes"]
    out = {}
    for v in names:
        out[v] = {"median_ms_per_gate": 1e3 * statistics.median(times[v]), "min_ms_per_gate": 1e3 * min(times[v]),
                  "passes": passes[v]}
        print(f"{v:22s} median {out[v]['median_ms_per_gate']:.4f} ms/gate  min {out[v]['min_ms_per_gate']:.4f}  "
              f"passes {passes[v]}", flush=True)
    print(json.dumps({"qubits": n, "gates": len(circ.gates), "variants": out}))
    assert abs(reg.total_prob() - 1) < 1e-9


if __name__ == "__main__":
    main()
