#!/bin/bash
# GPU box: DRAM-side counters of the wave kernel's memory path against the
# unfused streaming kernel on the same bytes.  One
# rocprofv3 --pmc run per counter group (at most 4 TCC counters a run) of
# bench.py --no-extras --seed 7 with QUEST_WAVE_NOOPS=1 (every wave pass
# memory-only) -- its timed window's passes and its unfused-gate reference
# (mat2DirectKernel, median of 5) -- summed per kernel by tools/pmc_mem.py.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_mem
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
i=0
for c in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
         "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
         "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  QUEST_WAVE_NOOPS=1 timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/g$i -o run --output-format csv -- \
      python3 $R/bench.py --no-extras --seed 7 --steps 20 --warmup 5 > $OUT/g$i.log 2>&1 || echo "group $i failed: $c"
done
python3 $R/tools/pmc_mem.py $OUT > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
