#!/bin/bash
# Round-6 placement (spare space capped at one array, re and im both placed
# by a probe of 1024 scattered ranges, the choice remembered per size):
# createQureg times of five 30-qubit registers in one process, then the
# seed-7 window in N fresh processes.
set -o pipefail
timeout -k 10 120 python - <<'PY' 2>&1
import time, quest_amd as qa
e = qa.Env()
regs = []
for i in range(5):
    t0 = time.perf_counter(); r = qa.Register(e, 30); r.sync(); dt = time.perf_counter() - t0
    st = qa.capi.getQuESTStats()
    print(f"createQureg(30) #{i}: {1e3*dt:.1f} ms, placement probes so far {st['placementProbes']}", flush=True)
    regs.append(r)
PY
for i in $(seq ${N:-8}); do
  QUEST_ALLOC_VERBOSE=1 timeout -k 10 120 python bench.py --no-extras --seed 7 --steps 20 --warmup 5 > gpurun_out/pl.json 2> gpurun_out/pl.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/pl.json')); print('process $i seed 7', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
  grep "GiB arrays" gpurun_out/pl.err | head -1 | cut -c1-150
done
