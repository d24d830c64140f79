#!/bin/bash
# Small registers: the window's planning latency (26 / 28 qubits, 10 layers,
# five seeds) under front-flush thresholds.
set -o pipefail
for q in 26 28; do
  for ff in 600 384 256 128; do
    QUEST_FRONT_FLUSH=$ff timeout -k 10 120 python bench.py --no-extras --qubits $q --steps 10 --warmup 3 > gpurun_out/ff.json 2> gpurun_out/ff.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ff.json')); c=d['config']; print('q$q ff$ff', '%.4g'%(d['value']*1e6), 'us/gate', c['passes'], 'passes', [round(s['window_ms'],2) for s in c['seeds']])"
  done
done
