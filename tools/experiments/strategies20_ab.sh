#!/bin/bash
# 20 search strategies from 30 local qubits (new default) vs 16, headline bench, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2 3; do
  for e in "X=1" "QUEST_PLAN_STRATEGIES=16"; do
    env $e timeout -k 10 240 python bench.py --no-extras > gpurun_out/s20_bench.json 2>> gpurun_out/strategies20_ab.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/s20_bench.json').read().strip().splitlines()[-1]); print('$e', '%.5g'%(d['value']*1e3), 'ms/gate', d['config']['passes'], [round(s['s_per_gate']*1e3,4) for s in d['config']['seeds']], [s['passes'] for s in d['config']['seeds']])" | tee -a gpurun_out/strategies20_ab.txt
  done
done
