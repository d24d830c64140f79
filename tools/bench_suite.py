#!/usr/bin/env python3
"""Every benchmark configuration named in BASELINE.json, on one GPU:

  tutorial    3-qubit tutorial circuit (plumbing; P(|111>), P(q2=1))
  sweep       single-qubit-gate time vs #qubits (the headline metric, unfused:
              one hadamard = one pass over the state), n = 20..34, targets
              low / middle / high
  random30    30-qubit fp64 depth-30 random layered circuit (fused)
  fork30      the fork's exact 30-qubit benchmark program (490 gates,
              30 calcProbOfOutcome, 10 getAmp; tutorial_example.c), wall time
              vs its published 3783.93 s estimate
  q34         34 qubits (256 GiB state, one MI355X): single gates + 6 layers
  qft30       30-qubit quantum Fourier transform on |+>^n (result |0>)
  density17   17-qubit density matrix (also 2^34 amplitudes) + damping on
              every qubit + gates

    python tools/bench_suite.py [--only sweep,fork30] [--max-qubits 34] [--out f.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quest_amd.utils.bench_workloads import (run_density17, run_fork30, run_q34, run_qft30,  # noqa: E402
                                             run_random30, run_sweep, run_tutorial)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="tutorial,sweep,random30,qft30,fork30,q34,density17")
    ap.add_argument("--max-qubits", type=int, default=34)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import quest_amd as qa
    from quest_amd.ops import capi

    env = qa.Env()
    res = {"backend": capi.getQuESTBackend(), "precision": capi.getQuEST_PREC()}
    todo = args.only.split(",")
    if "tutorial" in todo:
        run_tutorial(env, res)
    # the 30-qubit programs first: after the sweep frees 256 GiB, the next
    # allocation pays the driver's page clearing on first touch
    if "fork30" in todo:
        run_fork30(env, res)
    if "random30" in todo:
        run_random30(env, res)
    if "qft30" in todo:
        run_qft30(env, res)
    if "sweep" in todo:
        run_sweep(env, res, args.max_qubits)
    if "q34" in todo and args.max_qubits >= 34:
        run_q34(env, res)
    if "density17" in todo and args.max_qubits >= 34:
        run_density17(env, res)
    text = json.dumps(res, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
