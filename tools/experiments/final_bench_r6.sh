#!/bin/bash
# GPU box, end of round 6: the full single-GPU bench (all extras) and rocprofv3
# kernel statistics of the headline bench (no extras).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6_final.json 2> gpurun_out/bench_r6_final.err || exit $?
tail -c 600 gpurun_out/bench_r6_final.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r6_final -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --steps 20 --warmup 5 > $R/gpurun_out/prof_r6_final.log 2>&1 || exit $?
tail -1 $R/gpurun_out/prof_r6_final.log | cut -c1-300
