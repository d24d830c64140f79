#!/bin/bash
# PMC passes over the wave micro-benchmark's op-heavy workloads (one pass per
# counter group, tools/experiments/wave_micro.py --only); results under gpurun_out/pmcm
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcm
mkdir -p $O
rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
W="$R/tools/experiments/wave_micro.py --qubits 28 --reps 1 --only ${ONLY:-heavy|mid}"
timeout -k 10 120 python3 $W > $O/micro.txt 2>&1 || exit $?
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
           "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_MISSES" \
           "SQ_IFETCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $W > $O/p$i.log 2>&1 || echo "pass $i rc=$?" >> $O/status.txt
done
python3 $R/tools/pmc_summary.py $O > $O/summary.txt 2>&1 || true
