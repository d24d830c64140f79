#!/bin/bash
# Full flushes the strategy search plans, with no front flush before them
# (10-layer windows below 600 ops): search first (QUEST_PLAN_SEARCH_SPLIT=0)
# vs the first pass at once and the search over the rest while it runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for e in 1 0; do
    QUEST_PLAN_SEARCH_SPLIT=$e timeout -k 10 200 python3 tools/experiments/sweep_ab.py --sizes 27 28 29 30 --tag "split=$e" \
      >> $R/gpurun_out/search_split_ab.txt 2> $R/gpurun_out/search_split_ab.err || exit $?
    tail -1 $R/gpurun_out/search_split_ab.txt
  done
done
for q in 28 30; do
  rm -f $R/gpurun_out/wts$q.trace
  QUEST_TRACE=$R/gpurun_out/wts$q.trace timeout -k 10 120 python3 tools/experiments/window_timeline.py --qubits $q \
    > $R/gpurun_out/wts$q.txt 2>&1 || exit $?
  grep seed $R/gpurun_out/wts$q.txt | cut -c1-220
done
