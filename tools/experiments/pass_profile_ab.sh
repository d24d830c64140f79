#!/bin/bash
# pass_profile.sh twice on one box: normal, and with QUEST_WAVE_NOOPS=1
# (the same passes' loads and stores only): per-pass op cost vs memory floor
R=$GRAFT_REPO_ROOT
bash $R/tools/pass_profile.sh && mv $R/gpurun_out/pp $R/gpurun_out/pp_ops &&
QUEST_WAVE_NOOPS=1 bash $R/tools/pass_profile.sh && mv $R/gpurun_out/pp $R/gpurun_out/pp_noops &&
python3 - <<'PY'
import os
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/"
def rows(d):
    out = []
    for l in open(R + d + "/passes.txt"):
        p = l.split()
        if p and p[0].replace('.', '', 1).isdigit() and len(p) > 5:
            out.append((float(p[0]), p[1], int(p[2]), int(p[3]), int(p[4]), l[l.index('['):].strip()))
    return out
a, b = rows("pp_ops"), rows("pp_noops")
with open(R + "pass_ab.txt", "w") as f:
    f.write(f"{'ops_ms':>7} {'mem_ms':>7} {'extra':>6} {'wops':>5} {'tr':>4}  positions > 12\n")
    for x, y in zip(a, b):
        f.write(f"{x[0]:7.3f} {y[0]:7.3f} {x[0]-y[0]:6.3f} {x[3]:5d} {x[4]:4d}  {x[5]}\n")
    f.write(f"total ops {sum(x[0] for x in a):.1f} ms, memory-only {sum(y[0] for y in b):.1f} ms\n")
PY
