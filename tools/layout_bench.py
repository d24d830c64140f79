#!/usr/bin/env python3
"""Cost of reads across qubit layouts (GPU box): two 30-qubit registers after
different 20-layer random circuits (relabelling passes leave each in its own
qubit layout), then

  * calcInnerProduct of the two (permuted kernel: one pass over both, no
    relayout; QUEST_PERM_KERNELS=0: both registers relaid out first),
  * canonicaliseQureg of one (relabelling wave passes; QUEST_RELAYOUT_PASSES=0:
    SWAP ops on the LDS kernel),
  * one unfused Hadamard for scale (one streaming pass).

    python tools/layout_bench.py [--qubits 30] [--layers 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--layers", type=int, default=20)
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    a, b = qa.Register(env, n), qa.Register(env, n)
    for r, seed in ((a, 3), (b, 4)):
        r.init_plus()
        random_layered(n, args.layers, seed=seed).apply(r)
        r.sync()
    la, lb = capi.getQubitLayout(a.q), capi.getQubitLayout(b.q)
    out = {"qubits": n, "moved_a": sum(1 for i, p in enumerate(la) if i != p),
           "moved_b": sum(1 for i, p in enumerate(lb) if i != p),
           "perm_kernels": os.environ.get("QUEST_PERM_KERNELS", "1"),
           "relayout_passes": os.environ.get("QUEST_RELAYOUT_PASSES", "1"),
           "perm_tile_bits": os.environ.get("QUEST_PERM_TILE_BITS", "11")}
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        ip = a.inner(b)
        ts.append(time.perf_counter() - t0)
    out["inner_ms"] = [round(1e3 * t, 3) for t in ts]
    out["inner"] = [ip.real, ip.imag]
    # same registers, same layout: the plain streaming inner product
    t0 = time.perf_counter()
    a.inner(a)
    out["inner_same_layout_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
    capi.resetQuESTStats()
    t0 = time.perf_counter()
    capi.canonicaliseQureg(b.q)
    b.sync()
    out["canonicalise_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
    out["canonicalise_passes"] = capi.getQuESTStats()["passes"]
    capi.setGateFusion(0)
    a.sync()
    t0 = time.perf_counter()
    a.h(n // 2)
    a.sync()
    out["unfused_h_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
