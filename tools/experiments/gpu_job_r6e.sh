#!/bin/bash
# round-6: SQ counters of the looping-grid kernel (one rocprofv3 --pmc pass over
# the headline bench) and the multi-rank bench tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    -d $R/gpurun_out/prof_r6_pmc -o run --output-format csv -- python3 $R/bench.py --no-extras --steps 5 --warmup 2 \
    > $R/gpurun_out/prof_r6_pmc.log 2>&1 || exit $?
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_bench.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/gpu_r6e.txt 2>&1
rc=$?; tail -6 gpurun_out/gpu_r6e.txt; exit $rc
