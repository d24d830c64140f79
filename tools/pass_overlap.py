#!/usr/bin/env python3
"""Compare the per-pass times of tools/pass_overlap.sh's three runs (full,
compute only, memory only): per pass T, C, M, and how T sits between
max(C, M) (perfect overlap) and C + M (none).

    python tools/pass_overlap.py gpurun_out/po
"""
import sys


def rows(path):
    out = []
    for line in open(path):
        f = line.split()
        if len(f) >= 7 and f[1] in ("wave", "lds", "direct"):
            out.append((float(f[0]), f[1], int(f[2]), int(f[3]), int(f[4]), float(f[5])))
    return out


def main():
    d = sys.argv[1]
    full, nomem, noops = (rows(f"{d}/{v}/passes.txt") for v in ("full", "nomem", "noops"))
    n = min(len(full), len(nomem), len(noops))
    print(f"{'pass':>4} {'engine':>6} {'ops':>4} {'wops':>5} {'tr':>4} {'T':>7} {'C':>7} {'M':>7} {'max':>7} {'C+M':>7} "
          f"{'ovl':>5} {'cyc':>6} {'C/cyc':>6}")
    tot = [0.0] * 5
    for i in range(n):
        T, eng, ops, wops, tr, cyc = full[i]
        C, M = nomem[i][0], noops[i][0]
        mx, sm = max(C, M), C + M
        ovl = (sm - T) / min(C, M) if min(C, M) > 0 else 0   # 1: fully hidden, 0: serial
        for k, v in enumerate((T, C, M, mx, sm)):
            tot[k] += v
        # C per 10^4 modeled cycles: how well the planner's cost model tracks the kernel
        rate = 1e4 * C / cyc if cyc else 0
        print(f"{i:4d} {eng:>6} {ops:4d} {wops:5d} {tr:4d} {T:7.3f} {C:7.3f} {M:7.3f} {mx:7.3f} {sm:7.3f} {ovl:5.2f} "
              f"{cyc:6.0f} {rate:6.2f}")
    T, C, M, mx, sm = tot
    print(f"sum  T {T:.2f}  C {C:.2f}  M {M:.2f}  sum max(C,M) {mx:.2f}  C+M {sm:.2f} ms; "
          f"T / sum max = {T / mx:.3f}")


if __name__ == "__main__":
    main()
