#!/usr/bin/env python3
"""Summary of a bench.py output file (the JSON line is the last line starting
with '{'; extras print progress lines before it).

    python tools/bench_summary.py gpurun_out/bench.json
"""
import json
import sys


def load(path):
    lines = [ln for ln in open(path) if ln.startswith("{")]
    return json.loads(lines[-1])


def main():
    d = load(sys.argv[1])
    c = d["config"]
    print(f"value {d['value'] * 1e3:.4f} ms/gate  n_gpus {d['n_gpus']}  passes {c['passes']} "
          f"({c.get('passes_per_seed', 0):.1f} per seed)  norm_err {c['norm_error']:.1e}")
    for r in c.get("seeds", []):
        extra = ""
        if "swap_ms" in r:
            extra = f"  swaps {r['swaps']} swap {r['swap_ms']:.2f} ms ({100 * r['swap_share']:.1f} %)"
        print(f"  seed {r['seed']:3d}: {r['s_per_gate'] * 1e3:.4f} ms/gate  {r['window_ms']:7.2f} ms  "
              f"{r['passes']} passes{extra}")
    for k in ("window1_s_per_gate", "unfused_gate_s", "extras_error"):
        if k in c:
            print(f"  {k}: {c[k]}")
    r = c.get("rotate29")
    if r:
        print(f"  rotate29: mean {r['mean_ms']:.3f} ms, fastest {r['fastest_ms']:.3f}, slowest {r['slowest_ms']:.3f}"
              f" (spread {r['spread']:.3f}), floor {r['bytes_per_gate'] / 6.29e12 * 1e3:.3f} ms at 6.29 TB/s")
    for k in ("fp32", "density17", "q34", "fork30"):
        if k in c:
            print(f"  {k}: {json.dumps(c[k])[:400]}")


if __name__ == "__main__":
    main()
