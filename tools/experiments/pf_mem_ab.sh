#!/bin/bash
# Memory-only passes (QUEST_WAVE_NOOPS=1) and full windows of the prefetch
# variants next to the default looping kernel, plus the unfused direct kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for v in default ${VARIANTS:-pf55 pf05 pf50}; do
  if [ $v = default ]; then unset QUEST_LIB; else export QUEST_LIB=$R/ab_libs/$v/libQuEST_hip_f64.so; fi
  for mode in noops full; do
    ( [ $mode = noops ] && export QUEST_WAVE_NOOPS=1
      timeout -k 10 150 python bench.py --no-extras --steps 20 --warmup 5 > gpurun_out/pm.json 2> gpurun_out/pm.err ) || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/pm.json')); c=d['config']
print('$v $mode', round(d['value']*1e3,4), 'ms/gate', c['passes'], 'passes; per pass %.3f ms; unfused gate %.3f ms' % (sum(s['window_ms'] for s in c['seeds'])/c['passes'], 1e3*c['unfused_gate_s']))"
  done
done
done
