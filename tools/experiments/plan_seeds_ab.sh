#!/bin/bash
# Candidate seeds per pass: 48 seeds / 32 distinct target sets (new default) vs 24 / 16 (before), headline bench interleaved,
# then the search-split GPU test.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2 3; do
  for e in "X=1" "QUEST_PLAN_SEEDS=24 QUEST_PLAN_TRIED=16"; do
    env $e timeout -k 10 240 python bench.py --no-extras > gpurun_out/ps_bench.json 2>> gpurun_out/plan_seeds_ab.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ps_bench.json').read().strip().splitlines()[-1]); print('$e', '%.5g'%(d['value']*1e3), 'ms/gate', d['config']['passes'], [round(s['s_per_gate']*1e3,4) for s in d['config']['seeds']], [s['passes'] for s in d['config']['seeds']])" | tee -a gpurun_out/plan_seeds_ab.txt
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 200 --timeout-method thread -k "split" > gpurun_out/split_test.txt 2>&1
rc=$?; tail -2 gpurun_out/split_test.txt; exit $rc
