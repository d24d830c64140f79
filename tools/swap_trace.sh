#!/bin/bash
# GPU box: kernel + memory-copy trace of the distributed swaps of two ranks
# sharing one GPU (IPC transport; COMM=rccl with QUEST_RCCL_SHARED_GPU=1:
# RCCL itself), then the per-swap overlap summary of tools/swap_trace.py.
# QUBITS local qubits per rank (default 28).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/swaptr
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/swaptr -o run_%pid% -- \
    python3 $R/tools/dist_bench.py --ranks 2 --qubits ${QUBITS:-28} --steps 6 --warmup 1 --comm ${COMM:-ipc} \
    > $R/gpurun_out/swaptr/run.log 2>&1 || exit $?
python3 $R/tools/swap_trace.py $R/gpurun_out/swaptr > $R/gpurun_out/swaptr/summary.txt 2>&1
