#!/bin/bash
# A/B/C... of the headline bench between environment settings on one box:
# bash tools/experiments/ab_env_multi.sh ROUNDS "VAR=a" "VAR=b" "VAR=c" ...
N=$1; shift
for r in $(seq $N); do
  for v in "$@"; do
    env $v timeout -k 10 120 python bench.py --no-extras --steps 20 --warmup 5 > gpurun_out/ab_env.json 2> gpurun_out/ab_env.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_env.json')); print('$v', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
  done
done
