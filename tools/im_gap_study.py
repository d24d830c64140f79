#!/usr/bin/env python3
"""Streaming rate of the unfused gate against the distance D between a
register's re and im arrays (one allocation, im QUEST_IM_GAP bytes after the
end of re): the reference's per-target benchmark (bench_workloads
run_rotate29: compactUnitary on every target, 20 synced trials) at n qubits
for several gaps, each in a child process (the gap is read at allocation).

    python tools/im_gap_study.py [--qubits 29] [--gaps-gib 8,12,28]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import quest_amd as qa
from quest_amd.utils.bench_workloads import run_rotate29
env = qa.Env()
res = {}
run_rotate29(env, res, n=int(sys.argv[2]), trials=int(sys.argv[3]))
print("JSON " + json.dumps(res["rotate29"]))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=29)
    ap.add_argument("--gaps-gib", default="8,12,28")
    ap.add_argument("--trials", type=int, default=10)
    args = ap.parse_args()
    n = args.qubits
    size_gib = 8 * (1 << n) / 2 ** 30
    for g in args.gaps_gib.split(","):
        env = dict(os.environ, QUEST_IM_GAP=str(int(float(g) * 2 ** 30)))
        p = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(n), str(args.trials)], env=env, capture_output=True,
                           text=True, timeout=600)
        if p.returncode != 0:
            print(f"gap {g} GiB: failed\n{p.stderr[-1500:]}")
            sys.exit(1)
        r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("JSON ")][-1][5:])
        tb = [x["TBps"] for x in r["per_target"]]
        print(f"n={n} array {size_gib:.0f} GiB, gap {g} GiB (D = {size_gib + float(g):.0f} GiB): mean {r['mean_ms']:.3f} ms, "
              f"TB/s min {min(tb):.2f} mean {sum(tb) / len(tb):.2f} max {max(tb):.2f}; per target "
              + " ".join(f"{t:.2f}" for t in tb), flush=True)


if __name__ == "__main__":
    main()
