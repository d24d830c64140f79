#!/usr/bin/env python3
"""Per-pass cost of the headline circuit: which tile position sets are slow.

Run (GPU box) under the kernel tracer, with the library's pass trace on:

    QUEST_TRACE=gpurun_out/pp/trace.jsonl rocprofv3 --kernel-trace --output-format csv \
        -d gpurun_out/pp -o run -- python3 tools/pass_profile.py run --qubits 30 --layers 25

then join the two (here or there):

    python3 tools/pass_profile.py join gpurun_out/pp

Every "pass" trace event (src/hip/backend_hip.hip runProgram: tile positions,
ops, engine) is paired in order with the gate-kernel dispatches of the trace
(qa_wave_tile, the LDS tile kernels, the direct kernels); the table lists each
pass's duration, its positions above 12, and the achieved HBM bandwidth.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GATE_KERNELS = ("qa_wave_tile", "tilePassKernel", "DirectKernel", "mat2LowKernel")


def run(args):
    import quest_amd as qa
    from quest_amd.models import random_layered

    env = qa.Env()
    n = args.qubits
    reg = qa.Register(env, n)
    reg.init_plus()
    random_layered(n, args.layers, seed=args.seed).apply(reg)
    reg.sync()
    print("passes", qa.capi.getQuESTStats()["passes"])
    reg.close()


def join(args):
    d = args.dir
    trace = [json.loads(l) for l in open(glob.glob(os.path.join(d, "**", "trace.jsonl"), recursive=True)[0])]
    passes = [e for e in trace if e.get("ev") == "pass"]
    kfile = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(kfile)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if any(g in r["Kernel_Name"] for g in GATE_KERNELS)]
    # (the one-workgroup wave launch of the backend's start-up check has no
    # pass event)
    while len(ks) > len(passes) and "qa_wave_tile" in ks[0]["Kernel_Name"] and \
            int(ks[0]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"]) < 50000:
        ks = ks[1:]
    if len(ks) != len(passes):
        print(f"warning: {len(ks)} gate kernels vs {len(passes)} pass events", file=sys.stderr)
    out = []
    for p, k in zip(passes, ks):
        ms = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e6
        n = p["qubits"]
        tb = 2 * 16 * (1 << n) / 1e12   # fp64 re+im read and write, TB
        hi = [x for x in p["pos"] if x > 12]
        out.append((ms, p["engine"], p["ops"], p.get("wave_ops", 0), p.get("wave_tr", 0), p.get("wave_cycles", 0), hi,
                    tb / (ms / 1e3)))
    print(f"{'ms':>7} {'engine':>6} {'ops':>4} {'wops':>5} {'tr':>4} {'cyc':>6} {'TB/s':>5}  positions > 12")
    for ms, eng, ops, wops, tr, cyc, hi, bw in out:
        print(f"{ms:7.3f} {eng:>6} {ops:4d} {wops:5d} {tr:4d} {cyc:6.0f} {bw:5.2f}  {hi}")
    tot = sum(o[0] for o in out)
    print(f"total {tot:.2f} ms over {len(out)} passes, mean {tot / max(1, len(out)):.3f} ms")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--qubits", type=int, default=30)
    r.add_argument("--layers", type=int, default=25)
    r.add_argument("--seed", type=int, default=7)
    j = sub.add_parser("join")
    j.add_argument("dir")
    args = ap.parse_args()
    run(args) if args.cmd == "run" else join(args)


if __name__ == "__main__":
    main()
