#!/usr/bin/env python3
"""Overlap of the wave kernel with RCCL's kernels in one rank's rocprofv3
kernel trace (tools/overlap_study.sh): per RCCL kernel interval, the time
qa_wave_tile kernels ran inside it.

    python tools/overlap_report.py gpurun_out/overlap/prof1/r0
"""
import csv
import glob
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    wave = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "qa_wave_tile" in r["Kernel_Name"])
    comm = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows
                  if "nccl" in r["Kernel_Name"].lower() and "AllReduce" not in r["Kernel_Name"])
    tot_comm = tot_ov = 0
    print(f"{len(wave)} wave kernels, {len(comm)} RCCL send/recv kernels")
    for s, e, name in comm:
        ov = sum(max(0, min(e, we) - max(s, ws)) for ws, we in wave)
        tot_comm += e - s
        tot_ov += ov
        if e - s > 1_000_000:
            print(f"  {name}: {(e - s) / 1e6:8.2f} ms, wave kernels inside it {ov / 1e6:8.2f} ms ({100 * ov / (e - s):.1f} %)")
    if tot_comm:
        print(f"RCCL kernel time {tot_comm / 1e6:.2f} ms, of which overlapped by wave passes {tot_ov / 1e6:.2f} ms "
              f"({100 * tot_ov / tot_comm:.1f} %)")


if __name__ == "__main__":
    main()
