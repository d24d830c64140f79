#!/bin/bash
# GPU box: host timeline of fused windows (tools/experiments/window_timeline.py)
# at 24 / 26 / 28 qubits, and one rocprofv3 kernel trace of the 26-qubit run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for q in 24 26 28; do
  rm -f $R/gpurun_out/wt$q.trace
  QUEST_TRACE=$R/gpurun_out/wt$q.trace timeout -k 10 120 python3 tools/experiments/window_timeline.py --qubits $q \
    > $R/gpurun_out/wt$q.txt 2>&1 || exit $?
  cat $R/gpurun_out/wt$q.txt
done
cd /tmp && export TMPDIR=/tmp
rm -f $R/gpurun_out/wtp26.trace
QUEST_TRACE=$R/gpurun_out/wtp26.trace timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/wt_prof -o run --output-format csv -- \
    python3 $R/tools/experiments/window_timeline.py --qubits 26 > $R/gpurun_out/wtp26.txt 2>&1 || exit $?
cat $R/gpurun_out/wtp26.txt
