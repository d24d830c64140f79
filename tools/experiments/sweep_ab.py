"""fused_sweep rows (five seeds, 3 + 10 layers) at the given sizes, one JSON
line: per size s/gate and passes (quest_amd.utils.bench_workloads).

    python tools/experiments/sweep_ab.py --sizes 20 22 24 26 28 30 --tag name
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[20, 22, 24, 26, 28, 30])
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.utils.bench_workloads import run_fused_sweep

    env = qa.Env()
    res = {}
    run_fused_sweep(env, res, sizes=tuple(args.sizes))
    print(json.dumps({"tag": args.tag, "rows": {r["n"]: [round(r["s_per_gate"] * 1e6, 3), r["passes"],
                                                          round(r["per_byte_vs_30q"] or 0, 3)]
                                                for r in res["fused_sweep"]}}), flush=True)


if __name__ == "__main__":
    main()
