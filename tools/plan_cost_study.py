#!/usr/bin/env python3
"""Modeled pass costs of the wave planner on the bench circuit, without a GPU
(host build, QUEST_PLAN_ONLY=1, tools/plan_study.py): for every setting and
circuit seed the pass count, the modeled compute of every pass (waveOpCycles
summed over the pass's wave ops, the planner's own cost model) and
sum(max(C, M)) with M = one pass's memory stream in the same units
(--score-mem, default 18000: the round-4 overlap study measured 3.6 ms of
compute per 10^4 modeled cycles and 6.7 ms per memory-only pass at 30
qubits, profiles/r4/overlap_study_r4b.txt).

    python tools/plan_cost_study.py [--seeds 7,1,2,3,4] [--set "name:ENV=V,ENV=V" ...]
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M = 18000.0


def run(seed, env_over, qubits, layers):
    env = dict(os.environ, QUEST_WAVE_DUMP="1", **env_over)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plan_study.py"), "--seed", str(seed),
                        "--qubits", str(qubits), "--layers", str(layers)],
                       env=env, capture_output=True, text=True, timeout=600)
    hdr = re.search(r"passes (\d+)", p.stdout)
    if not hdr:
        raise RuntimeError(p.stdout + p.stderr)
    P = int(hdr.group(1))
    cyc = [float(m.group(1)) for m in re.finditer(r"cycles (\d+)", p.stderr)][-P:]
    return P, cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="7,1,2,3,4")
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--layers", type=int, default=20)
    ap.add_argument("--score-mem", type=float, default=M, help="M of the score, in modeled cycles")
    ap.add_argument("--set", action="append", default=[],
                    help='"name:ENV=V,ENV=V" (default: the build default and the planner without cost hooks)')
    args = ap.parse_args()
    m = args.score_mem
    sets = args.set or ["default:", "nocost:QUEST_PLAN_MEM_CYCLES=0"]
    print(f"# {args.qubits} qubits, {args.layers} layers; M = {m:.0f} modeled cycles per pass")
    print(f"{'setting':24s} {'seed':>4s} {'passes':>6s} {'sumC':>8s} {'sumMax':>8s} {'maxC':>7s}")
    tot = {}
    for spec in sets:
        name, _, kv = spec.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        for seed in args.seeds.split(","):
            P, cyc = run(int(seed), env, args.qubits, args.layers)
            sm = sum(max(c, m) for c in cyc)
            t = tot.setdefault(name, [0, 0.0])
            t[0] += P
            t[1] += sm
            print(f"{name:24s} {seed:>4s} {P:6d} {sum(cyc):8.0f} {sm:8.0f} {max(cyc):7.0f}")
    for name, (P, sm) in tot.items():
        print(f"{name:24s} total passes {P}, sum max(C, M) {sm:.0f}")


if __name__ == "__main__":
    main()
