#!/bin/bash
# A/B/C of the headline bench between library builds on one box:
# bash tools/ab_libs_multi.sh ROUNDS default path/to/other.so ...   ("default" = the in-tree library)
N=$1; shift
for r in $(seq $N); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset QUEST_LIB; else export QUEST_LIB=$v; fi
    timeout -k 10 120 python bench.py --no-extras --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
  done
done
