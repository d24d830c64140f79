#!/bin/bash
# GPU box: per-pass durations of the headline bench (all windows, warm-ups included) joined with the
# planner's per-pass records (tools/pass_profile.py join): which passes run long and what they hold.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pp
rm -f $R/gpurun_out/pp/trace.jsonl
cd /tmp && export TMPDIR=/tmp
QUEST_TRACE=$R/gpurun_out/pp/trace.jsonl timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/pp -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --steps 20 --warmup 5 > $R/gpurun_out/pp/bench.log 2>&1 || exit $?
cd $R && python3 tools/pass_profile.py join gpurun_out/pp > gpurun_out/pp/join.txt 2>&1 || exit $?
tail -3 gpurun_out/pp/join.txt
