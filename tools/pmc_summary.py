#!/usr/bin/env python3
"""Table of rocprofv3 PMC counters per dispatch of one kernel, merged over
the passes of a directory tree (tools/experiments/pmc_micro.sh):

    python3 tools/pmc_summary.py gpurun_out/pmcm [--kernel qa_wave_tile]

Rows are the kernel's dispatches in order (the n-th dispatch of every pass
is the same workload), columns the counters of all passes."""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="qa_wave_tile")
    ap.add_argument("--sum", action="store_true", help="one row: every counter summed over the dispatches")
    args = ap.parse_args()
    table = defaultdict(dict)   # dispatch rank -> counter -> value
    names = []
    for f in sorted(glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True)):
        rows = [r for r in csv.DictReader(open(f)) if args.kernel in r["Kernel_Name"]]
        order = sorted({int(r["Dispatch_Id"]) for r in rows})
        rank = {d: i for i, d in enumerate(order)}
        for r in rows:
            c = r["Counter_Name"]
            if c not in names:
                names.append(c)
            table[rank[int(r["Dispatch_Id"])]][c] = table[rank[int(r["Dispatch_Id"])]].get(c, 0.0) + float(r["Counter_Value"])
    if args.sum:
        tot = {n: sum(table[k].get(n, 0.0) for k in table) for n in names}
        for n in names:
            print(f"{n:28s} {tot[n]:14.4e}")
        wc = tot.get("SQ_WAVE_CYCLES")
        if wc:
            for n in names:
                if n != "SQ_WAVE_CYCLES" and n != "SQ_BUSY_CYCLES":
                    print(f"{n + ' / wave cycles':42s} {tot[n] / wc:8.3f}")
        return
    print("dispatch " + " ".join(f"{n:>22s}" for n in names))
    for k in sorted(table):
        print(f"{k:8d} " + " ".join(f"{table[k].get(n, float('nan')):22.4e}" for n in names))


if __name__ == "__main__":
    main()
