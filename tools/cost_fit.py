#!/usr/bin/env python3
"""Fit the wave planner's per-handler cost model (waveOpCycles,
src/core/wave.cpp) to measured compute: per-pass compute-only kernel times
of tools/pass_overlap.sh runs (the --nomem kernel) against the handler mix of
the same passes, taken from the host planner's dump of the same circuit
(tools/plan_study.py --warmup 0: the plan is deterministic and identical to
the GPU's).  Least squares over handler groups; prints the fitted cycles
per op next to the model's.

    python tools/cost_fit.py gpurun_out/po:7 gpurun_out/po1:1 gpurun_out/po2:2 [--layers 25]
"""
import argparse
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL = {"M2": 600, "M2R": 300, "M2RI": 300, "D2S": 300, "ANTI": 450, "SWAP": 211, "DIAG": 256, "D2L": 300,
         "LM2R": 724, "LM2RI": 578, "LANTI": 600, "LSWAP": 425, "ROTY": 207, "ROTX": 207, "HADD": 140, "YSW": 250,
         "YSWC": 250, "DROT": 190, "DNEG": 61, "DMULI": 236, "DMULNI": 236, "DROTN": 259, "DSC": 128}
TRL = [517, 563, 341, 339, 264, 259]
GROUPS = ["MAT", "SWAP", "LSWAP", "LANE", "TR01", "TR25", "TRW", "ROT", "HADD", "DNEG", "PHASE"]


def group(h):
    k = h.split("_")[0]
    if k == "TR":
        lane = int(re.search(r"_l(\d)", h).group(1))
        return ("TR01" if lane < 2 else "TR25"), TRL[lane]
    if k == "TRW":
        return "TRW", 300
    c = MODEL.get(k, 300)
    if re.search(r"_c[12]$", h) and k not in ("LM2R", "LM2RI", "LANTI", "LSWAP"):
        c /= 2   # slot-controlled: the model halves per control bit (one bit assumed)
    if k in ("M2", "M2R", "M2RI", "ANTI", "D2S", "D2L", "YSW", "YSWC"):
        return "MAT", c
    if k in ("LM2R", "LM2RI", "LANTI"):
        return "LANE", c
    if k in ("ROTY", "ROTX"):
        return "ROT", c
    if k in ("SWAP", "LSWAP", "HADD", "DNEG"):
        return k, c
    return "PHASE", c


def passes_of(seed, layers):
    env = dict(os.environ, QUEST_WAVE_DUMP="2")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plan_study.py"), "--seed", str(seed),
                        "--layers", str(layers), "--warmup", "0"], env=env, capture_output=True, text=True,
                       timeout=600)
    out, cur = [], []
    for line in p.stderr.split("\n"):
        if line.startswith("H wh_"):
            cur.append(line[5:])
        elif line.startswith("wave pass:"):
            out.append(cur)
            cur = []
    return out


def measured(d):
    rows = []
    for line in open(os.path.join(d, "nomem", "passes.txt")):
        f = line.split()
        if len(f) >= 6 and f[1] == "wave":
            rows.append(float(f[0]))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("runs", nargs="+", help="dir:seed")
    ap.add_argument("--layers", type=int, default=25)
    args = ap.parse_args()
    X, y, M = [], [], []
    for spec in args.runs:
        d, seed = spec.rsplit(":", 1)
        hs = passes_of(int(seed), args.layers)
        ms = measured(d)
        if len(hs) != len(ms):
            print(f"{d}: {len(hs)} planned vs {len(ms)} measured passes; skipped", file=sys.stderr)
            continue
        for h, t in zip(hs, ms):
            cnt = dict.fromkeys(GROUPS, 0.0)
            mod = dict.fromkeys(GROUPS, 0.0)
            for x in h:
                g, c = group(x)
                cnt[g] += 1
                mod[g] += c
            X.append([cnt[g] for g in GROUPS])
            M.append([mod[g] for g in GROUPS])
            y.append(t)
    X, y, M = np.array(X), np.array(y), np.array(M)
    # time per op of each group (ms), non-negative least squares by clipping
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    model_ms = y.sum() / M.sum()          # ms per modeled cycle, overall
    print(f"{len(y)} passes; overall {1e4 * model_ms:.3f} ms per 10^4 modeled cycles")
    print(f"{'group':6s} {'ops':>6s} {'model cyc/op':>12s} {'fitted cyc/op':>13s}")
    for i, g in enumerate(GROUPS):
        n = X[:, i].sum()
        mc = M[:, i].sum() / n if n else 0
        print(f"{g:6s} {n:6.0f} {mc:12.0f} {coef[i] / model_ms:13.0f}")
    pred = X @ coef
    print("residual rms %.3f ms; model-only rms %.3f ms" % (np.sqrt(np.mean((y - pred) ** 2)),
                                                         np.sqrt(np.mean((y - M.sum(1) * model_ms) ** 2))))


if __name__ == "__main__":
    main()
