#!/bin/bash
# End of round 6: the full single-GPU bench (all extras), rocprofv3 kernel statistics of the headline bench, smoke()
# (the GPU suite: tools/experiments/gpu_suite_durations.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6_final.json 2> gpurun_out/bench_r6_final.err || exit $?
tail -c 300 gpurun_out/bench_r6_final.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r6_final -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --steps 20 --warmup 5 > $R/gpurun_out/prof_r6_final.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6.txt 2>&1 || { cat gpurun_out/smoke_r6.txt; exit 1; }
tail -1 gpurun_out/smoke_r6.txt
exit 0
