#!/bin/bash
# GPU box: round-5 evidence -- rocprofv3 kernel statistics of the headline
# bench (no extras), then one PMC pass of SQ counters over the same run.
# Results under gpurun_out/prof_r5*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r5 -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --steps 20 --warmup 5 > $R/gpurun_out/prof_r5.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    -d $R/gpurun_out/prof_r5_pmc -o run --output-format csv -- python3 $R/bench.py --no-extras --steps 5 --warmup 2 \
    > $R/gpurun_out/prof_r5_pmc.log 2>&1 || exit $?
