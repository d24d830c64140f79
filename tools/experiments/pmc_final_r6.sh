#!/bin/bash
# End of round 6: SQ counters of qa_wave_tile over the headline bench (one --pmc pass), final planner.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    -d $R/gpurun_out/prof_r6_pmc_final -o run --output-format csv -- python3 $R/bench.py --no-extras --steps 5 --warmup 2 \
    > $R/gpurun_out/prof_r6_pmc_final.log 2>&1 || exit $?
ls $R/gpurun_out/prof_r6_pmc_final
