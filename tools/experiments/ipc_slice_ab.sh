# IPC swap time vs exchange slice size: 2 ranks x 29 qubits sharing one GPU
# (tools/dist_bench.py), rank 0's per-swap host times
for mb in 256 1024 64 256 1024; do
  echo "slice_mb=$mb $(QUEST_EXCHANGE_SLICE_MB=$mb timeout -k 10 200 python tools/dist_bench.py --ranks 2 --qubits 29 --steps 6 --warmup 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["swaps"], [round(x,1) for x in d["swap_host_ms_rank0"]], round(d["s_per_gate"]*1e3,3))')" || exit $?
done
