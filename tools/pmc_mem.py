#!/usr/bin/env python3
"""Per-kernel means of the rocprofv3 counters of tools/pmc_mem.sh, per byte
of state traffic (wave passes and the unfused gate kernels each move the
whole 30-qubit state: 16 GiB read + 16 GiB written per dispatch).

    python tools/pmc_mem.py gpurun_out/pmc_mem
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sums = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> values per dispatch
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            kk = "wave" if "qa_wave_tile" in k else "direct" if "DirectKernel" in k else None
            if kk is None:
                continue
            key = (kk, r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
        for (kk, _, c), v in per.items():
            sums[kk][c].append(v)
    for kk in ("wave", "direct"):
        print(f"## {kk}: mean per dispatch")
        for c in sorted(sums[kk]):
            vs = sums[kk][c]
            print(f"  {c:36s} {sum(vs) / len(vs):16.4e}  ({len(vs)} dispatches)")


if __name__ == "__main__":
    main()
