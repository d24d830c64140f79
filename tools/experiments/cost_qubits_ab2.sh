#!/bin/bash
# Compute-aware trimming at 27-29 local qubits: QUEST_PLAN_COST_QUBITS 27 vs 30 (fused_sweep windows).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for c in 27 30; do
    QUEST_PLAN_COST_QUBITS=$c timeout -k 10 200 python3 tools/experiments/sweep_ab.py --sizes 27 28 29 --tag "cost_qubits=$c" \
      >> $R/gpurun_out/cost_qubits_ab2.txt 2> $R/gpurun_out/cost_qubits_ab2.err || exit $?
    tail -1 $R/gpurun_out/cost_qubits_ab2.txt
  done
done
