#!/bin/bash
# GPU box: round-6 evidence -- the full single-GPU bench (all extras), rocprofv3
# kernel statistics of the headline bench (no extras), and a kernel trace of
# a 26-qubit window (GPU busy time vs the window: the small-register overhead).
# Results under gpurun_out/prof_r6*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6.json 2> gpurun_out/bench_r6.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r6 -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --steps 20 --warmup 5 > $R/gpurun_out/prof_r6.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_r6_q26 -o run --output-format csv -- \
    python3 $R/bench.py --no-extras --qubits 26 --steps 10 --warmup 3 > $R/gpurun_out/prof_r6_q26.log 2>&1 || exit $?
