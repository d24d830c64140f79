#!/bin/bash
# The Python binding's per-gate fast path (src/py/gatecall.c) against the
# ctypes path: fused_sweep rows (us / gate, passes, per byte vs 30 qubits) and
# the headline bench, interleaved.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for gc in 1 0; do
    QUEST_PY_GATECALL=$gc timeout -k 10 240 python tools/experiments/sweep_ab.py --tag "gatecall=$gc" \
      >> gpurun_out/gatecall_ab.txt 2> gpurun_out/gatecall_ab.err || exit $?
    tail -1 gpurun_out/gatecall_ab.txt
  done
done
for ff in 256 128; do
  QUEST_FRONT_FLUSH=$ff timeout -k 10 240 python tools/experiments/sweep_ab.py --sizes 20 22 24 26 28 30 --tag "gatecall=1 ff=$ff" \
    >> gpurun_out/gatecall_ab.txt 2> gpurun_out/gatecall_ab.err || exit $?
  tail -1 gpurun_out/gatecall_ab.txt
done
for gc in 1 0; do
  QUEST_PY_GATECALL=$gc timeout -k 10 240 python bench.py --no-extras > gpurun_out/gc_bench.json 2>> gpurun_out/gatecall_ab.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/gc_bench.json')); print('bench gatecall=$gc', '%.5g'%(d['value']*1e3), 'ms/gate', d['config']['passes'], [round(s['s_per_gate']*1e3,4) for s in d['config']['seeds']])" | tee -a gpurun_out/gatecall_ab.txt
done
