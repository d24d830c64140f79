#!/bin/bash
# The headline bench three times in fresh processes on one box (final code).
set -o pipefail
for rep in 1 2 3; do
  timeout -k 10 240 python bench.py --no-extras > gpurun_out/rep_bench.json 2>> gpurun_out/final_repeat.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/rep_bench.json').read().strip().splitlines()[-1]); print('run $rep', '%.5g'%(d['value']*1e3), 'ms/gate', d['config']['passes'], [round(s['s_per_gate']*1e3,4) for s in d['config']['seeds']])" | tee -a gpurun_out/final_repeat.txt
done
