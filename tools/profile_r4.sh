#!/bin/bash
# Round-4 profile of the headline bench (GPU box): rocprofv3 kernel statistics
# of bench.py (20 timed layers, no extras), then the per-pass overlap study
# (full / compute-only / memory-only kernels, tools/pass_overlap.sh) of the
# 25-layer circuit of the round-3 study (profiles/r3/overlap_study_one_tile_per_wg.txt).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/bench.py --steps 20 --warmup 5 --no-extras"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o run --output-format csv -- $B \
    > $R/gpurun_out/prof_r4.log 2>&1 || exit $?
bash $R/tools/pass_overlap.sh || exit $?
python3 $R/tools/pass_overlap.py $R/gpurun_out/po > $R/gpurun_out/overlap_r4.txt 2>&1
