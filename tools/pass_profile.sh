#!/bin/bash
# GPU box: per-pass kernel times of the headline circuit joined with the
# library's pass trace (tools/pass_profile.py); output under gpurun_out/pp
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pp
QUEST_TRACE=$R/gpurun_out/pp/trace.jsonl timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
    -d $R/gpurun_out/pp -o run -- python3 $R/tools/pass_profile.py run --qubits ${QUBITS:-30} --layers ${LAYERS:-25} \
    > $R/gpurun_out/pp/run.log 2>&1 &&
python3 $R/tools/pass_profile.py join $R/gpurun_out/pp > $R/gpurun_out/pp/passes.txt 2>&1
