#!/bin/bash
# Instruction-cache and issue counters of the wave kernel on the headline
# bench; one rocprofv3 pass per group, summary in gpurun_out/pmci/summary.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmci
mkdir -p $O
B="$R/bench.py --steps 20 --warmup 5 --no-extras"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $B > $O/p$i.log 2>&1 || { echo "pass $i rc=$?" >> $O/status.txt; break; }
done
python3 - "$O" > $O/summary.txt <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "qa_wave_tile" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:14.4e}  ({len(n[k])} dispatches)")
PY
cat $O/summary.txt $O/status.txt 2>/dev/null
