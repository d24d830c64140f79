#!/bin/bash
# GPU box: idle gaps between the gate kernels of the headline bench's timed
# windows (is the host planner ever on the critical path?), with real passes
# and with memory-only passes (QUEST_WAVE_NOOPS=1: every pass at memory speed,
# the hardest case for the planner), under rocprofv3 --kernel-trace with the
# library's flush trace (plan_ms per flush).  Results: gpurun_out/gaps/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-full noops}; do
  mkdir -p $R/gpurun_out/gaps/$v
  unset QUEST_WAVE_NOOPS
  [ $v = noops ] && export QUEST_WAVE_NOOPS=1
  QUEST_TRACE=$R/gpurun_out/gaps/$v/trace.jsonl timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
      -d $R/gpurun_out/gaps/$v -o run -- python3 $R/bench.py --no-extras --steps 20 --warmup 5 ${SEEDARG:-} \
      > $R/gpurun_out/gaps/$v/bench.log 2>&1 || exit $?
  python3 $R/tools/gap_report.py $R/gpurun_out/gaps/$v > $R/gpurun_out/gaps/$v/gaps.txt 2>&1 || exit $?
done
