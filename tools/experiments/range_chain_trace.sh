#!/bin/bash
# GPU box: rank 0's kernel trace of the 2-rank RCCL-shared bench (26 qubits per rank, seeds 7 and 12) with one pass per swap
# range by range (QUEST_SWAP_RANGES_FIRST=1) and with the range-major chain of two (default): wave-kernel time inside the
# RCCL kernels (tools/overlap_report.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
ROUNDS=0 QUEST_SWAP_RANGES_FIRST=1 bash tools/overlap_study.sh > gpurun_out/chain_k1.txt 2>&1 || { tail -5 gpurun_out/chain_k1.txt; exit 1; }
cp gpurun_out/overlap/prof1_r0.txt gpurun_out/chain_k1_report.txt
ROUNDS=0 bash tools/overlap_study.sh > gpurun_out/chain_k2.txt 2>&1 || { tail -5 gpurun_out/chain_k2.txt; exit 1; }
cp gpurun_out/overlap/prof1_r0.txt gpurun_out/chain_k2_report.txt
tail -n 2 gpurun_out/chain_k1_report.txt gpurun_out/chain_k2_report.txt
