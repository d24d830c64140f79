#!/bin/bash
# Compute-only (nomem library) and full bench windows at 1 / 2 / 3 resident
# wave-tile workgroups per CU, static vs dynamic tile claims of looping
# grids: how much a pass's compute slows with fewer waves per SIMD (input to
# the double-buffered persistent kernel design).
set -o pipefail
R=$GRAFT_REPO_ROOT
for cfg in ${CFGS:-"full 0 1" "full 3 1" "full 3 0" "nomem 0 1" "nomem 3 1" "nomem 3 0" "nomem 2 1"}; do
  set -- $cfg
  lib=$1; wg=$2; dyn=$3
  ( [ $lib = nomem ] && export QUEST_LIB=$R/quest_amd/lib/var/nomem.so
    export QUEST_WAVE_WG_PER_CU=$wg QUEST_WAVE_DYNAMIC=$dyn
    timeout -k 10 150 python bench.py --no-extras --steps 20 --warmup 5 > gpurun_out/wg.json 2> gpurun_out/wg.err ) || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/wg.json')); c=d['config']
print('$lib wg$wg dyn$dyn', round(d['value']*1e3,4), 'ms/gate norm_err %.1e' % c.get('norm_error', -1), [ (s['seed'], round(s['window_ms'],1), s['passes']) for s in c['seeds']])"
done
