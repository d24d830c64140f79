#!/usr/bin/env python3
"""Host study of the search's pass-cost score: plan the bench's windows (30
qubits, 20 layers after 5, five seeds; QUEST_PLAN_ONLY) under the current
environment and price every planned pass with the hinge model fitted to
measured pass times, T = T0 + k * max(0, C - knee) (profiles/r6/pass_time_model.txt).

    QUEST_PLAN_SCORE_KNEE=11500 QUEST_PLAN_SCORE_SLOPE=0.76 python tools/experiments/score_study.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0, K, KNEE = 5.812, 0.000345, 11500


def main():
    arg = sys.argv[1] if len(sys.argv) > 1 else "7,11,12,13,17"
    if "-" in arg:
        a, b = arg.split("-")
        seeds = list(range(int(a), int(b) + 1))
    else:
        seeds = [int(s) for s in arg.split(",")]
    tot_p, tot_t = 0, 0.0
    out = []
    procs = {}
    par = int(os.environ.get("STUDY_JOBS", "4"))
    pending = list(seeds)
    traces = {}
    while pending or procs:
        while pending and len(procs) < par:
            sd = pending.pop(0)
            tr = f"/tmp/score_study_{os.getpid()}_{sd}.trace"
            if os.path.exists(tr):
                os.remove(tr)
            env = dict(os.environ, QUEST_TRACE=tr, QUEST_TRACE_PASS_CYCLES="1")
            procs[sd] = subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "plan_study.py"), "--seed",
                                          str(sd)], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            traces[sd] = tr
        for sd in list(procs):
            if procs[sd].poll() is not None:
                assert procs[sd].returncode == 0, sd
                del procs[sd]
        if procs:
            import time
            time.sleep(0.05)
    for sd in seeds:
        tr = traces[sd]
        evs = [json.loads(line) for line in open(tr)]
        os.remove(tr)
        # the timed window: the passes after the warm-up's last flush (plan_study resets stats there)
        flushes = [i for i, e in enumerate(evs) if e["ev"] == "flush"]
        cyc = [e["wave_cycles"] for e in evs if e["ev"] == "pass"]
        p = [e for e in evs if e["ev"] == "pass"]
        # warm-up passes: those of flushes before the window; plan_study's first flush is the warm-up's
        n_warm = evs[flushes[0]]["passes"] if flushes else 0
        win = [c for c in cyc[n_warm:]]
        t = sum(T0 + K * max(0.0, c - KNEE) for c in win)
        out.append((sd, len(win), round(t, 2)))
        tot_p += len(win)
        tot_t += t
    print(json.dumps({"passes": tot_p, "predicted_ms": round(tot_t, 2), "seeds": out}))


if __name__ == "__main__":
    main()
