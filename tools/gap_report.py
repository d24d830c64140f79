#!/usr/bin/env python3
"""GPU idle time between the gate kernels of each timed bench window
(tools/gap_study.sh output: a rocprofv3 kernel trace and the library's
QUEST_TRACE flush events).  A window is the run of gate kernels between two
host syncs; per window: kernels, span, busy time, the largest gaps, and the
plan_ms of its flushes.

    python tools/gap_report.py gpurun_out/gaps/noops
"""
import csv
import glob
import json
import os
import sys

GATE = ("qa_wave_tile", "tilePassKernel", "DirectKernel")


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:30]) for r in rows
          if any(g in r["Kernel_Name"] for g in GATE)]
    # windows: split where the gap exceeds 2 ms (a host sync / register switch)
    wins, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - cur[-1][1] > 2_000_000:
            wins.append(cur)
            cur = []
        cur.append(k)
    wins.append(cur)
    big = [w for w in wins if len(w) >= 8]
    print(f"{len(ks)} gate kernels in {len(wins)} groups; {len(big)} groups of >= 8 passes (the bench windows)")
    worst = 0.0
    for i, w in enumerate(big):
        busy = sum(e - s for s, e, _ in w)
        span = w[-1][1] - w[0][0]
        gaps = sorted(((w[j + 1][0] - w[j][1]) / 1e6 for j in range(len(w) - 1)), reverse=True)
        worst = max(worst, gaps[0] if gaps else 0)
        print(f"window {i}: {len(w)} passes, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms "
              f"({100 * busy / span:.2f} %), largest gaps {', '.join(f'{g:.3f}' for g in gaps[:4])} ms, "
              f"mean pass {busy / len(w) / 1e6:.3f} ms")
    print(f"largest inter-pass gap inside any window: {worst:.3f} ms")
    tr = os.path.join(d, "trace.jsonl")
    if os.path.exists(tr):
        fl = [json.loads(x) for x in open(tr) if '"flush"' in x]
        full = [e for e in fl if e.get("passes", 0) > 1 and e.get("ops", 0) > 200]
        for e in full:
            host = e["plan_ms"] - e.get("wait_ms", 0)
            print(f"full flush: {e['ops']} ops -> {e['passes']} passes, plan_ms {e['plan_ms']:.2f} of which "
                  f"waiting for the GPU {e.get('wait_ms', 0):.2f} and strategy search {e.get('search_ms', 0):.2f}: "
                  f"host planning {host:.2f} ms = {host / e['passes']:.2f} per pass")


if __name__ == "__main__":
    main()
