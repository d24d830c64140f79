#!/bin/bash
# Per-pass PMC counters of the headline bench's wave passes (one rocprofv3
# pass per counter group; tools/pmc_summary.py joins them per dispatch)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcb
mkdir -p $O
B="$R/bench.py --steps 5 --warmup 1 --no-extras"
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $B > $O/p$i.log 2>&1 || echo "pass $i rc=$?" >> $O/status.txt
done
python3 $R/tools/pmc_summary.py $O > $O/summary.txt 2>&1 || true
