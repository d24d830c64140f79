#!/bin/bash
# Run the framework's programs on N GPUs of ONE node, one rank per GPU over
# RCCL (xGMI) -- the counterpart of the reference's job scripts
# (examples/submissionScripts/mpi_SLURM_unit_tests.sh, mpi_SLURM_example.sh),
# without MPI: ranks find each other through RANK / WORLD_SIZE / LOCAL_RANK /
# MASTER_ADDR / MASTER_PORT (src/comm/bootstrap.cpp).
#
#   tools/run_node.sh N [bench] [fork] [golden]      (default: all three)
#
#   bench   python -m torch.distributed.run ... bench.py --gpus N
#           (30 qubits per GPU, the headline JSON line)
#   fork    the fork's 490-gate program (examples/random_circuit_benchmark.c,
#           C, one process per GPU) on the 30-qubit circuit
#   golden  the reference's golden unit suite (python -m quest_amd.utils.golden)
#           on N ranks
#
# Environment knobs: SHARED=1 puts every rank on GPU 0 (QUEST_RCCL_SHARED_GPU=1:
# RCCL over its network transport -- the one-GPU rehearsal of the data path;
# pair it with QUBITS=<= 30 - log2 N); QUBITS (qubits per GPU, default 30);
# STEPS / WARMUP (bench); PORT (MASTER_PORT, default 29500); OUT (log dir,
# default gpurun_out/run_node).  Every step has its own time limit; a failing
# step ends the script with its exit status.
set -u
N=${1:?usage: tools/run_node.sh N [bench] [fork] [golden]}
shift
WHAT=${*:-bench fork golden}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
QUBITS=${QUBITS:-30}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
PORT=${PORT:-29500}
OUT=${OUT:-gpurun_out/run_node}
mkdir -p "$OUT"
case $N in 1|2|4|8|16) ;; *) echo "N must be a power of two (1..16)" >&2; exit 2 ;; esac

export QUEST_BACKEND=hip
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MASTER_ADDR=127.0.0.1
export MASTER_PORT=$PORT
if [ "${SHARED:-0}" = 1 ]; then
    export QUEST_RCCL_SHARED_GPU=1 QUEST_COMM=rccl QUEST_COMM_TIMEOUT=${QUEST_COMM_TIMEOUT:-300}
    export HIP_VISIBLE_DEVICES=0
fi
LOG2N=0; while [ $((1 << LOG2N)) -lt "$N" ]; do LOG2N=$((LOG2N + 1)); done

# N processes of one command, ranks 0..N-1, wait for all; the exit status is
# the first nonzero one
launch() {
    local secs=$1; shift
    local pids=() rc=0
    for ((r = 0; r < N; r++)); do
        RANK=$r WORLD_SIZE=$N LOCAL_RANK=$r timeout -k 10 "$secs" "$@" > "$OUT/$STEP.$r.log" 2>&1 &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait "$p" || { s=$?; [ $rc = 0 ] && rc=$s; }; done
    return $rc
}

for STEP in $WHAT; do
    start=$(date +%s)
    case $STEP in
        bench)
            timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
                --master-addr 127.0.0.1 --master-port "$PORT" bench.py --gpus "$N" --qubits "$QUBITS" \
                --steps "$STEPS" --warmup "$WARMUP" > "$OUT/bench.log" 2>&1
            rc=$?
            grep '^{"metric"' "$OUT/bench.log" > "$OUT/bench_n$N.json"
            ;;
        fork)
            make -s build/examples/random_circuit_benchmark_hip > "$OUT/fork.build.log" 2>&1 || exit $?
            launch 900 build/examples/random_circuit_benchmark_hip examples/data/fork_circuit_30q.txt \
                $((QUBITS + LOG2N)) "$OUT/probs.dat" "$OUT/stateVector.dat"
            rc=$?
            ;;
        golden)
            launch 900 python -m quest_amd.utils.golden --log "$OUT/golden"
            rc=$?
            ;;
        *) echo "unknown step $STEP" >&2; exit 2 ;;
    esac
    echo "=== $STEP on $N rank(s): rc=$rc, $(( $(date +%s) - start )) s"
    [ "$STEP" = bench ] && cat "$OUT/bench_n$N.json"
    [ "$STEP" = fork ] && tail -3 "$OUT/fork.0.log"
    [ "$STEP" = golden ] && tail -2 "$OUT/golden.0.log"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
