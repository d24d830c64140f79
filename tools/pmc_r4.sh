#!/bin/bash
# Round-4 PMC passes of the headline bench's wave passes (GPU box), one
# counter group per run (rocprofv3 does not split counters over passes):
#   A: SQ issue / occupancy counters, B: HBM read bytes (FETCH_SIZE),
#   C: HBM write bytes (WRITE_SIZE).  Summaries: tools/pmc_summary.py --sum.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/bench.py --no-extras --steps 20 --warmup 5"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU \
    -d $R/gpurun_out/pmc4_a -o run --output-format csv -- $B > $R/gpurun_out/pmc4_a.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc4_b -o run --output-format csv -- $B > $R/gpurun_out/pmc4_b.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc4_c -o run --output-format csv -- $B > $R/gpurun_out/pmc4_c.log 2>&1
