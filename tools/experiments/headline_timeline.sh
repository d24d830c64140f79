#!/bin/bash
# GPU box: host timeline (window_timeline.py) and kernel gaps of the headline
# windows (30 qubits, 20 layers after 5, five seeds).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -f $R/gpurun_out/wth30.trace
QUEST_TRACE=$R/gpurun_out/wth30.trace timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/wt_prof_h30 -o run --output-format csv -- \
    python3 $R/tools/experiments/window_timeline.py --qubits 30 --layers 20 --warmup 5 > $R/gpurun_out/wth30.txt 2>&1 || exit $?
grep seed $R/gpurun_out/wth30.txt | cut -c1-300
cd $R && python3 tools/experiments/gpu_gaps.py gpurun_out/wt_prof_h30
