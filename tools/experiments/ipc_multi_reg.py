#!/usr/bin/env python3
"""Distributed numerics with several registers (run under torchrun, e.g. 8
IPC ranks sharing one GPU): R registers of n qubits, each gets its own random
layered window, one after another (like bench.py's seeds); after every window
the norm of every register is printed (rank 0), so a swap that writes into
the wrong register or races shows up where it happens.

    python -m torch.distributed.run --nproc-per-node 8 ... tools/experiments/ipc_multi_reg.py --regs 3
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regs", type=int, default=3)
    ap.add_argument("--local", type=int, default=22)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import math
    import quest_amd as qa
    from quest_amd.models import random_layered

    env = qa.Env()
    n = args.local + int(round(math.log2(env.num_ranks)))
    regs = []
    for i in range(args.regs):
        r = qa.Register(env, n)
        r.init_plus()
        regs.append(r)
    for rnd in range(args.rounds):
        for i, r in enumerate(regs):
            random_layered(n, args.layers, seed=100 * rnd + i).apply(r)
            r.sync()
            errs = [abs(x.total_prob() - 1.0) for x in regs]
            if env.rank == 0:
                print(f"round {rnd} after register {i}: norm errors " + " ".join(f"{e:.1e}" for e in errs), flush=True)
    st = qa.capi.getQuESTStats()
    if env.rank == 0:
        print(f"swaps {st['swaps']} passes {st['passes']}", flush=True)


if __name__ == "__main__":
    main()
