#!/bin/bash
# Instruction counts of the wave kernel on the headline bench (driver
# config), one rocprofv3 pass; summary in gpurun_out/pmc3/summary.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc3
mkdir -p $O
B="$R/bench.py --steps 20 --warmup 5 --no-extras"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
    -d $O/p1 -o run --output-format csv -- python3 $B > $O/p1.log 2>&1 || exit $?
python3 - "$O" > $O/summary.txt <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "qa_wave_tile" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
waves = tot.get("SQ_WAVES", 1)
tiles_waves = waves  # one wave = one slice of every tile it processes
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:14.4e}  ({len(n[k])} dispatches)")
PY
cat $O/summary.txt
