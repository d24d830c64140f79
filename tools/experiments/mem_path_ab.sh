#!/bin/bash
# GPU box: memory-only wave passes (QUEST_WAVE_NOOPS=1: loads + stores, no ops)
# of the bench window under the wave-grid knobs, against the same run's
# unfused gate (the direct streaming kernel).  Two interleaved rounds.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/mem_path_ab.txt
: > $OUT
for round in 1 2; do
  for v in "" "QUEST_WAVE_TILE_MAP=1" "QUEST_WAVE_WG_PER_CU=2" "QUEST_WAVE_WG_PER_CU=3" "QUEST_WAVE_WG_PER_CU=4"; do
    line=$(env QUEST_WAVE_NOOPS=1 $v timeout -k 10 120 python3 $R/bench.py --no-extras --steps 20 --warmup 5) || exit $?
    echo "$line" | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); c=d['config']
print(f'round $round  {\"$v\" or \"default\":26s} window {d[\"ms_per_step\"]*20:8.2f} ms  passes {c[\"passes\"]}  per pass {d[\"ms_per_step\"]*20/c[\"passes\"]:6.3f} ms  unfused gate {1e3*c[\"unfused_gate_s\"]:6.3f} ms')
" >> $OUT || exit $?
  done
done
cat $OUT
