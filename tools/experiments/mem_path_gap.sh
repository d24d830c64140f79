#!/bin/bash
# GPU box: the bench window's passes per pass, memory only (QUEST_WAVE_NOOPS=1)
# and with ops, at the default re/im distance and at D = 16 GiB (the round-4
# placement), against the same run's unfused gate.  Two interleaved rounds.
#   SEEDS="7,12" VARIANTS="ENV=V ENV=V;ENV=V" bash tools/experiments/mem_path_gap.sh
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/mem_path_gap.txt
: > $OUT
for round in 1 2; do
  IFS=';' read -ra VS <<< "${VARIANTS:-QUEST_WAVE_NOOPS=1;QUEST_WAVE_NOOPS=1 QUEST_IM_GAP=8589934592;QUEST_WAVE_NOOPS=0;QUEST_WAVE_NOOPS=0 QUEST_IM_GAP=8589934592}"
  for v in "${VS[@]}"; do
    line=$(env $v timeout -k 10 150 python3 $R/bench.py --no-extras --seeds ${SEEDS:-7,12} --steps 10 --warmup 3) || exit $?
    echo "$line" | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); c=d['config']
per=' '.join(f'{s[\"seed\"]}:{s[\"window_ms\"]/s[\"passes\"]:.3f}' for s in c['seeds'])
print(f'round $round  {\"$v\":44s} ms/pass {per}  passes {c[\"passes\"]}  unfused gate {1e3*c[\"unfused_gate_s\"]:6.3f} ms')
" >> $OUT || exit $?
  done
done
cat $OUT
