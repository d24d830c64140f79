#!/bin/bash
# Compute-aware trimming below 27 local qubits (QUEST_PLAN_COST_QUBITS 22 default vs 27): its host time
# (a wave lowering per candidate pass) against the passes it shortens; plus the planner's host profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for c in 22 27; do
    QUEST_PLAN_COST_QUBITS=$c timeout -k 10 200 python3 tools/experiments/sweep_ab.py --sizes 22 23 24 25 26 --tag "cost_qubits=$c" \
      >> $R/gpurun_out/cost_qubits_ab.txt 2> $R/gpurun_out/cost_qubits_ab.err || exit $?
    tail -1 $R/gpurun_out/cost_qubits_ab.txt
  done
done
for q in 24 26; do
  QUEST_PLAN_PROFILE=1 timeout -k 10 120 python3 tools/experiments/sweep_ab.py --sizes $q --tag prof 2>&1 | grep -E "plan profile|rows" | tee -a $R/gpurun_out/cost_qubits_ab.txt
done
