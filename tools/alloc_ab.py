#!/usr/bin/env python3
"""Does the placement of a register's re / im arrays change the streaming
rate?  Registers with different placements (QUEST_ALLOC_MODE / QUEST_IM_OFFSET,
read at allocation) live side by side; rounds alternate between them: the
headline workload (20 layers of bench.py's circuit, one window) and unfused H
on qubits 0 and n/2.

    python tools/alloc_ab.py [--qubits 30] [--rounds 3] [--reverse]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

G = 1 << 30
# (label, QUEST_ALLOC_MODE, QUEST_IM_OFFSET, QUEST_ALLOC_PAD) -- sizes for 30 qubits (8 GiB arrays)
PLACEMENTS = [("split (default) #1", 0, 0, 0), ("contiguous #1", 2, 0, 0), ("split (default) #2", 0, 0, 0),
              ("contiguous #2", 2, 0, 0), ("split (default) #3", 0, 0, 0), ("contiguous #3", 2, 0, 0)]
if os.environ.get("ALLOC_AB_SET") == "distance":
    # joint allocations, im starting D GiB after re (QUEST_IM_OFFSET = D - array size);
    # ALLOC_AB_ARRAY_GIB = the array size (8 at 30 qubits), ALLOC_AB_D = the distances
    _a = float(os.environ.get("ALLOC_AB_ARRAY_GIB", "8"))
    _ds = [float(x) for x in os.environ.get("ALLOC_AB_D", "8,12,16,20,32,8,16").split(",")]
    PLACEMENTS = [(f"joint, im {d:g} GiB after re", 1, int((d - _a) * G), 0) for d in _ds]
if os.environ.get("ALLOC_AB_SET") == "vmm":
    # mode 3: one reserved address range, physical memory mapped for re and
    # im only, im QUEST_IM_DIST bytes after re (this set sizes for 30 qubits)
    PLACEMENTS = [("split (default)", 0, 0, 0), ("joint, im 16 GiB after re", 1, 8 * G, 0),
                  ("vmm, im 16 GiB after re", 3, 16 * G, 0), ("vmm, im 8 GiB after re", 3, 8 * G, 0),
                  ("vmm, im 32 GiB after re", 3, 32 * G, 0), ("vmm, im 16 GiB after re #2", 3, 16 * G, 0),
                  ("split (default) #2", 0, 0, 0)]
if os.environ.get("ALLOC_AB_SET") == "offsets":
    PLACEMENTS = [("split (default)", 0, 0, 0), ("joint, im 24 GiB after re", 1, 24 * G, 0),
                  ("split, each in a 32 GiB alloc", 0, 0, 24 * G), ("joint in a 48 GiB alloc", 1, 0, 32 * G),
                  ("joint, im 8 GiB after re", 1, 8 * G, 0), ("split (default), later", 0, 0, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reverse", action="store_true", help="allocate in reverse order")
    args = ap.parse_args()
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.models.circuits import Circuit
    from quest_amd.ops import capi

    n = args.qubits
    env = qa.Env()
    circ = random_layered(n, 25, seed=7)
    chunks, i = [], 0
    for layer in range(25):
        cnt = n + len(range(layer % 2, n - 1, 2))
        chunks.append(circ.gates[i:i + cnt])
        i += cnt
    warm = Circuit(n, [g for c in chunks[:5] for g in c])
    timed = Circuit(n, [g for c in chunks[5:] for g in c])
    regs = []
    order = PLACEMENTS[::-1] if args.reverse else PLACEMENTS
    for label, mode, off, pad in order:
        os.environ["QUEST_ALLOC_MODE"] = str(mode)
        os.environ["QUEST_IM_OFFSET"] = str(off)
        os.environ["QUEST_IM_DIST"] = str(off)
        os.environ["QUEST_ALLOC_PAD"] = str(pad)
        r = qa.Register(env, n)
        r.init_plus()
        warm.apply(r)
        r.sync()
        regs.append((label, r))
    os.environ["QUEST_ALLOC_MODE"] = "0"
    os.environ["QUEST_ALLOC_PAD"] = "0"
    res = {label: {"layered": [], "h0": [], "hmid": []} for label, _ in regs}

    def clock(r, fn):
        r.sync()
        t0 = time.perf_counter()
        fn()
        r.sync()
        return time.perf_counter() - t0

    for _ in range(args.rounds):
        for label, r in regs:
            res[label]["layered"].append(clock(r, lambda: timed.apply(r)) / len(timed.gates))
            capi.setGateFusion(0)
            for key, t in (("h0", 0), ("hmid", n // 2)):
                clock(r, lambda: r.h(t))
                res[label][key].append(min(clock(r, lambda: r.h(t)) for _ in range(3)))
            capi.setGateFusion(1)
    print(f"n={n}: best of {args.rounds} rounds; layered = ms/gate of the bench's 20 timed layers")
    for label, _ in regs:
        d = res[label]
        print(f"{label:28s} layered {1e3 * min(d['layered']):.4f}  H(0) {1e3 * min(d['h0']):.3f} ms  "
              f"H(n/2) {1e3 * min(d['hmid']):.3f} ms", flush=True)
    for _, r in regs:
        r.close()


if __name__ == "__main__":
    main()
