cd $GRAFT_REPO_ROOT
for n in 2 4 8; do
  rm -f gpurun_out/tr_$n.*
  QUEST_COMM=ipc OMP_NUM_THREADS=1 QUEST_TRACE=$GRAFT_REPO_ROOT/gpurun_out/tr_$n.txt timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2957$n bench.py --gpus $n --steps 20 --warmup 5 --allow-transport > gpurun_out/scale_ipc_$n.log 2>&1 || exit $?
  grep -h '"rank": 0' gpurun_out/tr_$n.txt | grep -E '"swap"|"flush"' | cut -c1-160 > gpurun_out/tr_${n}_r0.txt
  grep '^{' gpurun_out/scale_ipc_$n.log | cut -c1-400
done
