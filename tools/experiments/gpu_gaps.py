#!/usr/bin/env python3
"""GPU idle time between the gate kernels of a rocprofv3 kernel trace (the
bench's timed window: are passes back to back, or does the host planner
starve the GPU?).

    python tools/experiments/gpu_gaps.py gpurun_out/bt [--last N]
"""
import csv
import glob
import os
import sys

GATE = ("qa_wave_tile", "tilePassKernel", "DirectKernel")


def main():
    d = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows
          if any(g in r["Kernel_Name"] for g in GATE)]
    if last:
        ks = ks[-last:]
    busy = sum(e - s for s, e, _ in ks)
    span = ks[-1][1] - ks[0][0]
    gaps = [(ks[i + 1][0] - ks[i][1], i) for i in range(len(ks) - 1)]
    print(f"{len(ks)} gate kernels, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %)")
    for g, i in sorted(gaps, reverse=True)[:8]:
        print(f"  gap {g / 1e6:7.3f} ms after kernel {i} ({ks[i][2]}, {(ks[i][1] - ks[i][0]) / 1e6:.3f} ms)")


if __name__ == "__main__":
    main()
