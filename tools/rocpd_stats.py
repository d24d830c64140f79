#!/usr/bin/env python3
"""Per-kernel statistics (calls, total / mean / min / max ns) from a rocprofv3
SQLite result (the default output format of rocprofv3 in ROCm 7):

    python tools/rocpd_stats.py gpurun_out/prof_final/run_results.db [--dispatches qa_wave_tile]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--dispatches", default=None, help="also list every dispatch of kernels matching this name")
    args = ap.parse_args()
    cur = sqlite3.connect(args.db).cursor()
    rows = list(cur.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                            "max(vgpr_count), max(lds_size) from kernels group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'mean_ms':>9s} {'min_ms':>8s} {'max_ms':>8s} {'%':>6s}")
    for name, n, tot, avg, mn, mx, vg, lds in rows:
        print(f"{name[:70]:70s} {n:6d} {tot / 1e6:10.3f} {avg / 1e6:9.3f} {mn / 1e6:8.3f} {mx / 1e6:8.3f} "
              f"{100 * tot / total:6.2f}")
    if args.dispatches:
        print(f"\ndispatches of {args.dispatches} (ms, in order):")
        d = [r[0] / 1e6 for r in cur.execute("select duration from kernels where name like ? order by start",
                                             (f"%{args.dispatches}%",))]
        print(" ".join(f"{x:.2f}" for x in d))


if __name__ == "__main__":
    main()
