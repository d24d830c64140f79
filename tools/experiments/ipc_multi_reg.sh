#!/bin/bash
# $1 name, rest env
name=$1; shift
port=$((29500 + RANDOM % 2000))
( for kv in "$@"; do export "$kv"; done
  QUEST_COMM=ipc QUEST_BACKEND=hip OMP_NUM_THREADS=1 timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=${RANKS:-8} \
   --master-addr 127.0.0.1 --master-port $port tools/experiments/ipc_multi_reg.py ${ARGS:-} 2> gpurun_out/imr_$name.err | sed "s/^/$name: /" )
