#!/usr/bin/env python3
"""Density-matrix channel timings at n qubits (2n-qubit state): damping,
dephasing and two-qubit dephasing on every qubit (pair), one sync each.
Run with QUEST_DEPHASE_DIAG=0 / 1 to compare the dephasing lowerings.

    python tools/dephase_ab.py [--qubits 16]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=16)
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    d = qa.Register(env, n, density=True)
    d.init_plus()
    d.sync()
    out = {}
    for name, fn, cnt in (("damping", lambda: [d.damping(q, 0.1) for q in range(n)], n),
                          ("dephase", lambda: [d.dephase(q, 0.1) for q in range(n)], n),
                          ("dephase2", lambda: [d.dephase2(q, q + 1, 0.1) for q in range(0, n - 1, 2)], n // 2),
                          ("depolarise2", lambda: [d.depolarise2(q, q + 1, 0.1) for q in range(0, n - 1, 2)], n // 2)):
        best = 1e9
        for _ in range(2):
            capi.resetQuESTStats()
            d.sync()
            t0 = time.perf_counter()
            fn()
            d.sync()
            best = min(best, (time.perf_counter() - t0) / cnt)
        out[name] = (best, capi.getQuESTStats()["passes"])
    mode = os.environ.get("QUEST_DEPHASE_DIAG", "1")
    tq = os.environ.get("QUEST_TILE_QUBITS", "default")
    print(f"density n={n} QUEST_DEPHASE_DIAG={mode} QUEST_TILE_QUBITS={tq}: " +
          ", ".join(f"{k} {1e3 * v[0]:.2f} ms/channel ({v[1]} passes)" for k, v in out.items()) +
          f", trace {d.total_prob():.12f}", flush=True)
    d.close()


if __name__ == "__main__":
    main()
