#!/bin/bash
# GPU box: overlapped qubit swaps on one GPU with 2 RCCL ranks sharing it
# (QUEST_RCCL_SHARED_GPU=1: RCCL's network transport over loopback, the only
# RCCL path a one-GPU box has).  The bench window with QUEST_SWAP_OVERLAP=1 and
# =0 (same box, interleaved), then one run of each rank under rocprofv3
# --kernel-trace so the timeline shows qa_wave_tile next to the RCCL kernels.
#   QUBITS (per rank, default 26), SEEDS (default 7,12), ROUNDS (default 2)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
Q=${QUBITS:-26}
OUT=$R/gpurun_out/overlap
mkdir -p $OUT
run2() {   # $1 = tag, $2 = overlap 0/1, $3 = profile dir ("" = none)
  local port=$((29500 + RANDOM % 2000))
  local pids=""
  for r in 0 1; do
    local pre=""
    [ -n "$3" ] && pre="rocprofv3 --kernel-trace --output-format csv -d $3/r$r -o run --"
    RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$port QUEST_COMM=rccl \
      QUEST_RCCL_SHARED_GPU=1 QUEST_COMM_TIMEOUT=150 QUEST_SWAP_OVERLAP=$2 OMP_NUM_THREADS=1 \
      timeout -k 10 200 $pre python3 $R/bench.py --gpus 2 --qubits $Q --steps 20 --warmup 5 --seeds ${SEEDS:-7,12} \
      > $OUT/$1.r$r.out 2> $OUT/$1.r$r.err &
    pids="$pids $!"
  done
  local rc=0
  for p in $pids; do wait $p || rc=$?; done
  return $rc
}
for i in $(seq ${ROUNDS:-2}); do
  for v in 1 0; do
    run2 "ov${v}_$i" $v "" || exit $?
    python3 $R/tools/bench_summary.py $OUT/ov${v}_$i.r0.out | sed "s/^/overlap=$v round $i: /"
  done
done
run2 prof1 1 $OUT/prof1 || exit $?
python3 $R/tools/overlap_report.py $OUT/prof1/r0 > $OUT/prof1_r0.txt 2>&1
cat $OUT/prof1_r0.txt
