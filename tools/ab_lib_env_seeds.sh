#!/bin/bash
# Same-box A/B of bench.py over environment variants on a given seed list:
#   SEEDS=14,15,16 bash tools/ab_lib_env_seeds.sh ROUNDS "name|lib.so|VAR=x VAR2=y" ...   (lib "" = in-tree)
N=$1; shift
for r in $(seq $N); do
  for spec in "$@"; do
    IFS='|' read name lib envs <<< "$spec"
    ( unset QUEST_LIB; [ -n "$lib" ] && export QUEST_LIB=$lib
      for kv in $envs; do export "$kv"; done
      timeout -k 10 150 python bench.py --no-extras --steps 20 --warmup 5 --seeds ${SEEDS:-7,11,12,13,17} > gpurun_out/ab.json 2> gpurun_out/ab.err ) || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$name', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes', 'norm_err %.1e' % d['config']['norm_error'])"
  done
done
