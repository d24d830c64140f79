#!/bin/bash
# Program uploads between dependent wave passes: the runtime's copy engine
# choice (SDMA vs blit kernel) against the ~20 us gap between passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for e in "X=1" "HSA_ENABLE_SDMA=0" "GPU_FORCE_BLIT_COPY_SIZE=1024"; do
    env $e timeout -k 10 200 python3 tools/experiments/sweep_ab.py --sizes 22 24 26 28 --tag "$e" \
      >> $R/gpurun_out/upload_ab.txt 2> $R/gpurun_out/upload_ab.err || exit $?
    tail -1 $R/gpurun_out/upload_ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
HSA_ENABLE_SDMA=0 QUEST_TRACE=$R/gpurun_out/wtn26.trace timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/wt_prof_nosdma -o run --output-format csv -- \
    python3 $R/tools/experiments/window_timeline.py --qubits 26 > $R/gpurun_out/wtn26.txt 2>&1 || exit $?
grep seed $R/gpurun_out/wtn26.txt
