#!/usr/bin/env python3
"""Instruction mix of the wave kernel on a planned circuit, without a GPU:
the handler of every op (host planner, QUEST_WAVE_DUMP=2) weighted by the
instructions of that handler in the generated assembly.

    QUEST_WAVE_DUMP=2 python tools/plan_study.py 2> /tmp/ops.txt
    python tools/wave_cost.py /tmp/ops.txt [--asm build/wave_f64/wave_kernel.s] [--last N]

Counts are per wave and tile summed over the passes (the last N passes:
the timed window of plan_study); controlled handlers are counted as if every
register passed (an upper bound)."""
import argparse
import collections
import re


def issue_cycles(op, text):
    """Wave-cycles per SIMD of one VALU instruction on gfx950, measured by
    tools/isa_micro.hip (profiles/r2/isa_micro_gfx950.txt)."""
    if op.startswith("v_swap") or "permlane" in op:
        return 8.2
    if op.startswith("v_cndmask") and "vcc" in text:
        return 22.6
    if "f64" in op or "b64" in op or op.startswith("v_pk_") or "_dpp" in op or op.startswith("v_cndmask") \
            or op.startswith("v_bfi"):
        return 4.3
    return 2.7


def handler_costs(path):
    cost = collections.defaultdict(collections.Counter)
    cur = None
    for line in open(path):
        m = re.match(r"^(wh_\w+):", line)
        if m:
            cur = m.group(1)
            continue
        t = line.strip()
        if cur is None or not t or t.startswith(".") or t.startswith("//") or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            cost[cur]["valu_f64" if "f64" in op else "valu"] += 1
            cost[cur]["cycles"] += issue_cycles(op, t)
        elif op.startswith("s_"):
            cost[cur]["salu"] += 1
        elif op.startswith("ds_"):
            cost[cur]["lds"] += 1
    return cost


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ops")
    ap.add_argument("--asm", default="build/wave_f64/wave_kernel.s")
    ap.add_argument("--last", type=int, default=0, help="only the last N passes")
    args = ap.parse_args()
    cost = handler_costs(args.asm)
    passes, cur = [], []
    for line in open(args.ops):
        if line.startswith("H "):
            cur.append(line.split()[1])
        elif line.startswith("wave pass:"):
            passes.append(cur)
            cur = []
    if args.last:
        passes = passes[-args.last:]
    fam = collections.defaultdict(collections.Counter)
    n = collections.Counter()
    for ps in passes:
        for h in ps:
            f = re.sub(r"_(s|l|b|c|m|a)\d+", "", h)
            f = re.sub(r"^wh_TR$", "wh_TR", f)
            if h.startswith("wh_TR_"):
                f = "wh_TR_l" + h.split("_l")[1]
            fam[f].update(cost[h])
            n[f] += 1
    tot = collections.Counter()
    for f in fam:
        tot.update(fam[f])
    print(f"{len(passes)} passes; per pass (per wave and tile):")
    print(f"{'family':16s} {'ops':>6s} {'valu':>8s} {'f64':>8s} {'cycles':>8s} {'salu':>8s} {'lds':>6s}")
    for f in sorted(fam, key=lambda f: -fam[f]["cycles"]):
        c = fam[f]
        P = len(passes)
        print(f"{f:16s} {n[f] / P:6.1f} {c['valu'] / P:8.0f} {c['valu_f64'] / P:8.0f} {c['cycles'] / P:8.0f} "
              f"{c['salu'] / P:8.0f} {c['lds'] / P:6.0f}")
    P = len(passes)
    print(f"{'total':16s} {sum(n.values()) / P:6.1f} {tot['valu'] / P:8.0f} {tot['valu_f64'] / P:8.0f} "
          f"{tot['cycles'] / P:8.0f} {tot['salu'] / P:8.0f} {tot['lds'] / P:6.0f}")


if __name__ == "__main__":
    main()
