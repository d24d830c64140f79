"""Small registers: time consecutive windows of the bench circuit, one sync
per window, to separate one-time costs (kernel loading, first use of a
program slot) from the steady state.

    python tools/experiments/small_reg.py --qubits 10 12 --windows 5 --layers 20
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import quest_amd as qa  # noqa: E402
from quest_amd.models import random_layered  # noqa: E402
from quest_amd.models.circuits import Circuit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, nargs="+", default=[10, 12])
    ap.add_argument("--windows", type=int, default=5)
    ap.add_argument("--layers", type=int, default=20)
    args = ap.parse_args()
    env = qa.Env()
    for n in args.qubits:
        reg = qa.Register(env, n)
        reg.init_plus()
        circ = random_layered(n, args.windows * args.layers, seed=1)
        per = len(circ.gates) // args.windows
        times = []
        for w in range(args.windows):
            reg.sync()
            t0 = time.perf_counter()
            t_enq = None
            Circuit(n, circ.gates[w * per:(w + 1) * per]).apply(reg)
            t_enq = time.perf_counter() - t0
            reg.sync()
            times.append((time.perf_counter() - t0, t_enq))
        print(f"q {n}: " + "  ".join(f"{1e6 * t / per:.2f}us/gate(enq {1e6 * e / per:.2f})" for t, e in times),
              flush=True)
        reg.close()


if __name__ == "__main__":
    main()
