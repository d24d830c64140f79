"""Host timeline of fused windows at one size: per window, when the gates were
queued, when each pass was launched (QUEST_TRACE "pass" events, aligned by the
trace's CLOCK_MONOTONIC origin) and when the sync returned -- against the
passes' GPU time (run under rocprofv3 --kernel-trace for that).

    QUEST_TRACE=gpurun_out/wt.trace python tools/experiments/window_timeline.py --qubits 26
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=26)
    ap.add_argument("--layers", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seeds", default="7,11,12,13,17")
    ap.add_argument("--marks", default=None, help="write the windows' CLOCK_MONOTONIC [start, queued, end] here "
                    "(rocprofv3 kernel timestamps use the same clock: tools/experiments/window_busy.py)")
    args = ap.parse_args()
    path = os.environ.get("QUEST_TRACE")
    assert path and path not in ("1", "stderr"), "QUEST_TRACE=<file>"
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit

    n, nl = args.qubits, args.layers
    env = qa.Env()
    r = qa.Register(env, n)
    marks = []
    for sd in [int(s) for s in args.seeds.split(",")]:
        circ = random_layered(n, args.warmup + nl, seed=sd)
        per, i = [], 0
        for layer in range(args.warmup + nl):
            cnt = n + len(range(layer % 2, n - 1, 2))
            per.append(circ.gates[i:i + cnt])
            i += cnt
        r.init_plus()
        for w in range(args.warmup):
            Circuit(n, per[w]).apply(r)
        r.sync()
        t0 = time.monotonic()
        for w in range(args.warmup, args.warmup + nl):
            Circuit(n, per[w]).apply(r)
        t1 = time.monotonic()
        r.sync()
        t2 = time.monotonic()
        marks.append((sd, t0, t1, t2))
    r.close()
    if args.marks:
        with open(args.marks, "w") as f:
            json.dump([{"seed": sd, "start": t0, "queued": t1, "end": t2} for sd, t0, t1, t2 in marks], f)
    evs = [json.loads(line) for line in open(path)]
    mono = next(e["monotonic"] for e in evs if e["ev"] == "trace_start")
    for sd, t0, t1, t2 in marks:
        launches = [1e3 * (mono + e["t"] - t0) for e in evs if e["ev"] == "pass" and t0 <= mono + e["t"] <= t2]
        flushes = [(1e3 * (mono + e["t"] - t0), e["passes"], e["plan_ms"]) for e in evs
                   if e["ev"] == "flush" and t0 <= mono + e["t"] <= t2]
        print(f"seed {sd}: window {1e3 * (t2 - t0):.3f} ms, gates queued at {1e3 * (t1 - t0):.3f}, "
              f"pass launches at [{', '.join(f'{x:.3f}' for x in launches)}], "
              f"flush ends [{', '.join(f'{a:.3f} ({p} passes, plan {pm:.3f})' for a, p, pm in flushes)}]", flush=True)


if __name__ == "__main__":
    main()
