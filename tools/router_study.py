#!/usr/bin/env python3
"""Swap counts of the distributed router's policy on the bench circuit,
without any state: a model of router::flushLogical / planSwap (logical window,
commutation-respecting issue, rank-qubit diagonal / anti-diagonal gates that
need no data, all rank qubits swapped at once) for comparing victim policies.

    python tools/router_study.py --qubits 33 --ranks 8 --layers 40 [--window 1024]

Policies: "belady" (src/core/router.cpp planSwap: the local qubits whose first
locality-requiring use is furthest go out), "cone" (the local qubits whose
move to a rank position would block the fewest queued ops go out)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GENERAL = {"h", "rx", "ry"}
DIAG = {"z", "s", "t", "rz"}
ANTI = {"x", "y"}


def ops_of(n, layers, seed):
    from quest_amd.models import random_layered
    circ = random_layered(n, layers, seed=seed)
    out = []
    for g in circ.gates:
        name, qs = g.name, g.qubits
        if name == "cnot":
            out.append(("anti", (qs[1],), (qs[0],)))
        elif name in GENERAL:
            out.append(("gen", (qs[0],), ()))
        elif name in DIAG:
            out.append(("diag", (qs[0],), ()))
        elif name in ANTI:
            out.append(("anti", (qs[0],), ()))
        else:
            raise ValueError(name)
    return out


def placement(op, glob):
    kind, tg, ct = op
    if not any(t in glob for t in tg):
        return "local"
    if kind == "diag":
        return "rank"
    if kind == "anti" and all(c in glob for c in ct):
        return "rank"
    return "blocked"


def issue_round(lq, glob):
    rest, btg, btouch = [], set(), set()
    for op in lq:
        tg, touch = set(op[1]), set(op[1]) | set(op[2])
        if not (tg & btouch) and not (touch & btg) and placement(op, glob) != "blocked":
            continue
        rest.append(op)
        btg |= tg
        btouch |= touch
    return rest


def blocked_count(lq, glob):
    return len(issue_round(lq, glob))


def plan_swap(lq, glob, n, policy):
    INF = 1 << 30
    first = {q: INF for q in range(n)}
    for i, op in enumerate(lq):
        if op[0] == "diag" or (op[0] == "anti" and not op[2]):
            continue   # need no data on a rank qubit (targetsNeedLocal)
        for t in op[1]:
            first[t] = min(first[t], i)
    need0 = set(lq[0][1])
    inn = sorted(glob, key=lambda q: first[q])
    cands = [q for q in range(n) if q not in glob and q not in need0]
    k = len(glob)
    if policy == "belady":
        out = sorted(cands, key=lambda q: -first[q])[:k]
    else:
        # greedy: add the victim that keeps the most queued ops issuable
        out = []
        newglob = set()
        for _ in range(k):
            best, score = None, None
            for q in cands:
                if q in out:
                    continue
                g = newglob | {q}
                s = blocked_count(lq, g)
                if score is None or s < score or (s == score and first[q] > first[best]):
                    best, score = q, s
            out.append(best)
            newglob.add(best)
    return set(out)


def simulate(ops, n, g, window, per_layer, policy):
    glob = set(range(n - g, n))
    lq, swaps = [], 0

    def flush():
        nonlocal lq, glob, swaps
        while lq:
            lq = issue_round(lq, glob)
            if lq:
                glob = plan_swap(lq, glob, n, policy)
                swaps += 1

    for layer_ops in per_layer:
        for op in layer_ops:
            lq.append(op)
            if len(lq) >= window:
                flush()
    flush()
    return swaps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=33)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--layers", type=int, default=40)
    ap.add_argument("--window", type=int, default=1024)
    ap.add_argument("--seeds", type=int, default=3)
    args = ap.parse_args()
    n, g = args.qubits, args.ranks.bit_length() - 1
    for policy in ("belady", "cone"):
        tot = 0
        for seed in range(7, 7 + args.seeds):
            ops = ops_of(n, args.layers, seed)
            per, i = [], 0
            for layer in range(args.layers):
                cnt = n + len(range(layer % 2, n - 1, 2))
                per.append(ops[i:i + cnt])
                i += cnt
            tot += simulate(ops, n, g, args.window, per, policy)
        print(f"{policy:7s} qubits {n} ranks {args.ranks} layers {args.layers} window {args.window}: "
              f"{tot / args.seeds:.2f} swaps per run")


if __name__ == "__main__":
    main()
