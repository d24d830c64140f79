#!/bin/bash
# Strategy search at 24-26 local qubits (QUEST_PLAN_SEARCH_QUBITS 24 vs 27 default) now that the first pass runs during it.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for c in 24 27; do
    QUEST_PLAN_SEARCH_QUBITS=$c timeout -k 10 200 python3 tools/experiments/sweep_ab.py --sizes 24 25 26 --tag "search_qubits=$c" \
      >> $R/gpurun_out/search_qubits_ab.txt 2> $R/gpurun_out/search_qubits_ab.err || exit $?
    tail -1 $R/gpurun_out/search_qubits_ab.txt
  done
done
