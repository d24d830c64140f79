#!/bin/bash
# GPU box: where the waves of qa_wave_tile spend their cycles (issue, wait,
# VALU, SALU, LDS) on the headline bench, for library / occupancy variants:
#   bash tools/pmc_stall.sh name[:lib.so[:wg_per_cu]] ...
# e.g. full nomem:quest_amd/lib/var/nomem.so nomem1:quest_amd/lib/var/nomem.so:1
# One PMC pass per variant (8 SQ counters), summed over the kernel's dispatches
# by tools/pmc_summary.py --sum.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for spec in "$@"; do
  IFS=: read name lib wg <<< "$spec"
  unset QUEST_LIB QUEST_WAVE_WG_PER_CU
  [ -n "$lib" ] && export QUEST_LIB=$R/$lib
  [ -n "$wg" ] && export QUEST_WAVE_WG_PER_CU=$wg
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmcs/$name -o run --output-format csv -- \
      python3 $R/bench.py --no-extras --steps 20 --warmup 5 > $R/gpurun_out/pmcs/$name.log 2>&1 || exit $?
  echo "== $name"; python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcs/$name --sum || exit $?
done
