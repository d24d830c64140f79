#!/usr/bin/env python3
"""Overlap of the distributed swap pipeline from a rocprofv3 kernel +
memory-copy trace (tools/swap_trace.sh): per process, the pack / unpack
kernels (packBitsKernel) and the exchange copies (IPC copy kernel, or RCCL's
kernels), grouped into swaps (gaps
of > 2 ms between consecutive pack/copy events split swaps); for each swap
its span, the busy time of pack/unpack and of the copies, and how much of
the copy time ran concurrently with a pack/unpack kernel.

    python tools/swap_trace.py gpurun_out/swaptr
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def intervals(rows, key_start="Start_Timestamp", key_end="End_Timestamp"):
    return sorted((int(r[key_start]), int(r[key_end])) for r in rows)


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def overlap_len(a, b):
    """Length of (union a) intersect (union b)."""
    def merge(iv):
        out = []
        for s, e in sorted(iv):
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        return out
    A, B = merge(a), merge(b)
    i = j = tot = 0
    while i < len(A) and j < len(B):
        s, e = max(A[i][0], B[j][0]), min(A[i][1], B[j][1])
        if s < e:
            tot += e - s
        if A[i][1] < B[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d = sys.argv[1]
    kfiles = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    cfiles = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    per = defaultdict(lambda: {"k": [], "c": []})
    for f in kfiles:
        for r in csv.DictReader(open(f)):
            if "pack" in r["Kernel_Name"].lower():
                per[(f, r.get("Process_Id", "0"))]["k"].append(r)
    for f in cfiles:
        for r in csv.DictReader(open(f)):
            if "DEVICE_TO_DEVICE" in r.get("Direction", "").upper():
                per[(f.replace("memory_copy", "kernel"), r.get("Process_Id", "0"))]["c"].append(r)
    # IPC pulls by the library's copy kernel (QUEST_IPC_BLIT=0, the default)
    # and RCCL's send / recv kernels (QUEST_COMM=rccl)
    for f in kfiles:
        for r in csv.DictReader(open(f)):
            if "copyVecKernel" in r["Kernel_Name"] or "nccl" in r["Kernel_Name"].lower():
                per[(f, r.get("Process_Id", "0"))]["c"].append(r)
    for (f, pid), v in sorted(per.items()):
        ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "k") for r in v["k"]] + \
             [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "c") for r in v["c"]]
        ev.sort()
        swaps, cur = [], []
        for e in ev:
            if cur and e[0] - max(x[1] for x in cur) > 2_000_000:
                swaps.append(cur)
                cur = []
            cur.append(e)
        if cur:
            swaps.append(cur)
        print(f"process {pid} ({os.path.basename(f)}): {len(v['k'])} pack/unpack kernels, {len(v['c'])} copies")
        print(f"{'swap':>4} {'span ms':>8} {'pack+unpack busy':>17} {'copy busy':>10} {'copy under kernels':>19}")
        for i, s in enumerate(swaps):
            k = [(a, b) for a, b, t in s if t == "k"]
            c = [(a, b) for a, b, t in s if t == "c"]
            span = max(x[1] for x in s) - min(x[0] for x in s)
            ov = overlap_len(k, c) / max(1, union_len(c))
            print(f"{i:4d} {span / 1e6:8.2f} {union_len(k) / 1e6:17.2f} {union_len(c) / 1e6:10.2f} {100 * ov:18.0f}%")


if __name__ == "__main__":
    main()
