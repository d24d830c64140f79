#!/bin/bash
# GPU box: bench.py under torchrun with 8 IPC ranks sharing the GPU (22 local
# qubits), once per variant "name|lib|ENV=V ..." -- prints each run's
# norm_error and swap count (bisecting a distributed numerics regression).
R=$GRAFT_REPO_ROOT
cd $R
for spec in "$@"; do
  IFS='|' read name lib envs <<< "$spec"
  port=$((29500 + RANDOM % 2000))
  out=$( (unset QUEST_LIB RANK WORLD_SIZE LOCAL_RANK; [ -n "$lib" ] && export QUEST_LIB=$R/$lib
          for kv in $envs; do export "$kv"; done
          QUEST_COMM=ipc QUEST_BACKEND=hip OMP_NUM_THREADS=1 timeout -k 10 200 python3 -m torch.distributed.run \
            --nnodes=1 --nproc-per-node=${RANKS:-8} --master-addr 127.0.0.1 --master-port $port bench.py \
            --gpus ${RANKS:-8} --qubits 22 --steps 4 --warmup 1 --allow-transport ${BENCH_ARGS:-} 2> gpurun_out/bisect_$name.err) ) || \
    { echo "$name: run failed rc=$?"; exit 1; }
  echo "$out" | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); c=d['config']
print('$name', 'norm_error %.3g' % c['norm_error'], 'swaps', c['swaps'], 'passes', c['passes'])"
done
