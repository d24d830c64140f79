#!/bin/bash
# GPU box: tools/overlap_demo.py (windows whose pre-swap passes leave the swap's
# victim out) on 2 RCCL ranks sharing the GPU (QUEST_RCCL_SHARED_GPU=1),
# QUEST_SWAP_OVERLAP=1 vs 0 interleaved, then rank 0 and 1 under rocprofv3
# --kernel-trace with overlap on, and tools/overlap_report.py on rank 0.
#   QUBITS (per rank, default 26), WINDOWS (8), LAYERS (4), ROUNDS (2)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/overlap_demo
mkdir -p $OUT
run2() {   # $1 = tag, $2 = overlap 0/1, $3 = profile dir ("" = none)
  local port=$((29500 + RANDOM % 2000))
  local pids=""
  for r in 0 1; do
    local pre=""
    [ -n "$3" ] && pre="rocprofv3 --kernel-trace --output-format csv -d $3/r$r -o run --"
    RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$port QUEST_COMM=rccl \
      QUEST_RCCL_SHARED_GPU=1 QUEST_COMM_TIMEOUT=150 QUEST_SWAP_OVERLAP=$2 OMP_NUM_THREADS=1 \
      timeout -k 10 200 $pre python3 $R/tools/overlap_demo.py --qubits ${QUBITS:-26} --windows ${WINDOWS:-8} \
      --layers ${LAYERS:-4} > $OUT/$1.r$r.out 2> $OUT/$1.r$r.err &
    pids="$pids $!"
  done
  local rc=0
  for p in $pids; do wait $p || rc=$?; done
  return $rc
}
for i in $(seq ${ROUNDS:-2}); do
  for v in 1 0; do
    run2 "ov${v}_$i" $v "" || exit $?
    echo "overlap=$v round $i: $(cat $OUT/ov${v}_$i.r0.out)"
  done
done
run2 prof1 1 $OUT/prof1 || exit $?
echo "profiled (overlap=1): $(cat $OUT/prof1.r0.out)"
python3 $R/tools/overlap_report.py $OUT/prof1/r0 > $OUT/prof1_r0.txt 2>&1
cat $OUT/prof1_r0.txt
