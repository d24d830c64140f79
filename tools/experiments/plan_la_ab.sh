#!/bin/bash
# Candidate lookahead 0.3 + the pass-time-model score (new defaults) vs neither, headline bench, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2 3; do
  for e in "X=1" "QUEST_PLAN_LOOKAHEAD=0 QUEST_PLAN_SCORE_KNEE=0"; do
    env $e timeout -k 10 240 python bench.py --no-extras > gpurun_out/la_bench.json 2>> gpurun_out/plan_la_ab.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/la_bench.json').read().strip().splitlines()[-1]); print('$e', '%.5g'%(d['value']*1e3), 'ms/gate', d['config']['passes'], [round(s['s_per_gate']*1e3,4) for s in d['config']['seeds']], [s['passes'] for s in d['config']['seeds']])" | tee -a gpurun_out/plan_la_ab.txt
  done
done
