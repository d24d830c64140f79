#!/bin/bash
# PMC counters of the wave kernel on the headline bench (driver config),
# one rocprofv3 pass per group; summary per kernel in gpurun_out/pmc2/summary.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc2
mkdir -p $O
B="$R/bench.py --steps 20 --warmup 5 --no-extras"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $B > $O/p$i.log 2>&1 || echo "pass $i rc=$?" >> $O/status.txt
done
python3 - "$O" > $O/summary.txt <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "qa_wave_tile" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print("qa_wave_tile, bench.py --steps 20 --warmup 5 (sum over dispatches)")
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:14.4e}  ({len(n[k])} dispatches)")
if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
    print(f"HBM bytes read (FETCH_SIZE kB x 2 on gfx950, see guide) {2 * tot['FETCH_SIZE'] * 1024:.4e}, written {tot['WRITE_SIZE'] * 1024:.4e}")
if "SQ_INSTS_VALU" in tot and "GRBM_GUI_ACTIVE" in tot:
    print(f"VALU busy ~ 4 x INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) = {4 * tot['SQ_INSTS_VALU'] / (1024 * tot['GRBM_GUI_ACTIVE'] / 8):.2f}")
PY
