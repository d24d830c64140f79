#!/usr/bin/env python3
"""Headline benchmark: single-qubit-gate time on a random fp64 state-vector
circuit (BASELINE.json: "single-qubit-gate time (s) vs #qubits, fp64
state-vector; 1/2/4/8-GPU scaling").

Workload (weak scaling): QUBITS_PER_GPU (default 30) qubits per GPU, so N
GPUs simulate 30 + log2(N) qubits, one rank per GPU (torchrun), the state
sharded over ranks and exchanged with RCCL over xGMI.  One *step* = one layer
of a seeded random circuit: a random gate from {H, X, Y, Z, S, T, Rx, Ry, Rz}
on every qubit, then a brick layer of CNOTs (the fork benchmark's gate mix,
tutorial_example.c:29-518).  `value` = wall seconds per gate over the timed
steps (max over ranks), gates applied through the public API exactly as a
user would call them (hadamard(), rotateX(), controlledNot(), ...).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--qubits Q] [--eager]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_S_PER_OP = 3783.9266747315614 / 667  # fork's estimate, tutorial_example.c:1-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--qubits", type=int, default=30, help="qubits per GPU")
    ap.add_argument("--eager", action="store_true", help="disable gate fusion (one pass per gate)")
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args()

    from quest_amd.parallel import allreduce_max, barrier, init_distributed

    rank, world = init_distributed()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    import torch

    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())

    import quest_amd as qa
    from quest_amd.models import random_layered

    if args.eager:
        os.environ["QUEST_FUSION"] = "0"
    env = qa.Env()
    n = args.qubits + int(round(math.log2(world)))
    reg = qa.Register(env, n)
    reg.init_plus()

    layers = args.warmup + args.steps
    circ = random_layered(n, layers, seed=args.seed)
    per_layer = len(circ.gates) // layers if layers else 0
    # split into layers (each layer: n one-qubit gates + CNOT brick)
    layer_gates = []
    i = 0
    for layer in range(layers):
        cnt = n + len(range(layer % 2, n - 1, 2))
        layer_gates.append(circ.gates[i:i + cnt])
        i += cnt

    from quest_amd.models.circuits import Circuit

    def run_layer(idx):
        Circuit(n, layer_gates[idx]).apply(reg)

    for w in range(args.warmup):
        run_layer(w)
    reg.sync()
    qa.capi.resetQuESTStats()

    barrier()
    reg.sync()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    gates = 0
    for s in range(args.steps):
        run_layer(args.warmup + s)
        gates += len(layer_gates[args.warmup + s])
    reg.sync()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    barrier()
    elapsed = allreduce_max(time.perf_counter() - t0)
    stats = qa.capi.getQuESTStats()

    norm = reg.total_prob()  # sanity (outside the timed region)
    # for reference, outside the timed region: one unfused gate (= one full
    # streaming pass over the state), median of 5
    qa.capi.setGateFusion(0)
    singles = []
    for _ in range(5):
        reg.sync()
        t1 = time.perf_counter()
        reg.h(n // 2)
        reg.sync()
        singles.append(time.perf_counter() - t1)
    qa.capi.setGateFusion(1)
    unfused_gate_s = allreduce_max(sorted(singles)[2])
    s_per_gate = elapsed / max(gates, 1)
    result = {
        "metric": "single-qubit-gate time (s) vs #qubits, fp64 state-vector; 1/2/4/8-GPU scaling",
        "value": s_per_gate,
        "unit": "s/gate",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / max(args.steps, 1),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": s_per_gate / BASELINE_S_PER_OP,
        "dtype": "fp64",
        "data": "synthetic: |+>^n initial state, seeded random layered circuit",
        "config": {
            "model": f"random layered circuit (1q gate on every qubit + CNOT brick), {n} qubits",
            "qubits": n,
            "qubits_per_gpu": args.qubits,
            "global_batch": 1,
            "seq_len": 1 << n,
            "gates_per_step": gates / max(args.steps, 1),
            "parallelism": f"dp{world}: amplitude-sharded over {world} GPU(s), qubit swaps over RCCL",
            "transport": qa.capi.getQuESTTransport(),
            "fusion": not args.eager,
            "passes": stats["passes"],
            "swaps": stats["swaps"],
            "norm_error": abs(norm - 1.0),
            "unfused_gate_s": unfused_gate_s,
            "backend": qa.capi.getQuESTBackend(),
        },
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    reg.close()


if __name__ == "__main__":
    main()
