#!/bin/bash
# Same-box A/B over circuit seeds with bench.py's default window (depth 30):
#   bash tools/ab_seeds_default.sh "seed1 seed2 ..." "name|VAR=x ..." ...
SEEDS=$1; shift
for seed in $SEEDS; do
  for spec in "$@"; do
    IFS='|' read name envs <<< "$spec"
    ( for kv in $envs; do export "$kv"; done
      timeout -k 10 120 python bench.py --no-extras --seed $seed > gpurun_out/ab.json 2> gpurun_out/ab.err ) || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('seed $seed $name', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes', d['steps'], 'steps')"
  done
done
