#!/usr/bin/env python3
"""GPU busy time inside each timed window: window_timeline.py --marks JSON
(CLOCK_MONOTONIC seconds) against a rocprofv3 kernel trace (ns, same clock).

    python tools/experiments/window_busy.py gpurun_out/marks.json gpurun_out/prof_dir
"""
import csv
import glob
import json
import os
import sys


def main():
    marks = json.load(open(sys.argv[1]))
    f = glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f)))
    for m in marks:
        a, b = int(m["start"] * 1e9), int(m["end"] * 1e9)
        inside = [(max(s, a), min(e, b)) for s, e in ks if e > a and s < b]
        busy = sum(e - s for s, e in inside)
        first = inside[0][0] - a if inside else None
        idle_mid = (b - a) - busy - (first or 0)
        print(f"seed {m['seed']}: window {(b - a) / 1e6:.3f} ms, first kernel at {first / 1e6:.3f} ms, "
              f"busy {busy / 1e6:.3f} ms ({100 * busy / (b - a):.1f} %), idle after the first kernel {idle_mid / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
