#!/bin/bash
# Range-major chains of three passes (QUEST_SWAP_RANGES_FIRST=3): the swap / fuzz / distributed GPU tests and rank 0's
# kernel trace of the 2-rank RCCL-shared bench (wave time inside RCCL kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export QUEST_SWAP_RANGES_FIRST=3
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_fuzz_dist.py tests/test_distributed.py -m gpu -x -v -s \
    --timeout 300 --timeout-method thread -k "ranges or overlapped or fuzz or ipc or rccl" > gpurun_out/range_chain_k3_tests.txt 2>&1 || \
    { grep -E "per window|passed|failed|FAILED" gpurun_out/range_chain_k3_tests.txt | tail -20; exit 1; }
grep -E "per window|passed|failed" gpurun_out/range_chain_k3_tests.txt | tail -5
ROUNDS=0 bash tools/overlap_study.sh > gpurun_out/chain_k3.txt 2>&1 || { tail -5 gpurun_out/chain_k3.txt; exit 1; }
cp gpurun_out/overlap/prof1_r0.txt gpurun_out/chain_k3_report.txt
tail -n 2 gpurun_out/chain_k3_report.txt
