#!/bin/bash
# Swap ranges on the bench windows: 2 / 4 RCCL ranks sharing the GPU (25 local
# qubits each), per-seed overlapped passes, swaps, norm; then the GPU test.
set -o pipefail
for ranks in 2 4; do
  for rf in 1 0; do
    QUEST_SWAP_RANGES_FIRST=$rf QUEST_RCCL_SHARED_GPU=1 QUEST_COMM_TIMEOUT=150 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$ranks \
      --master-addr 127.0.0.1 --master-port $((29700 + ranks + 10 * rf)) bench.py --gpus $ranks --qubits 25 --steps 20 --warmup 5 --no-extras \
      > gpurun_out/rb.json 2> gpurun_out/rb.err || { tail -20 gpurun_out/rb.err; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/rb.json') if l.startswith('{')][0]); c=d['config']
print('ranks $ranks first_avoid $rf', '%.4g ms/gate' % (d['value']*1e3), c['passes'], 'passes, swaps', c['swaps'], 'norm %.1e' % c['norm_error'], [(s['seed'], s['passes'], s.get('overlapped_passes')) for s in c['seeds']])"
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "ranges" > gpurun_out/gpu_r6d.txt 2>&1; rc=$?
grep -E "per window|passed|failed|Error" gpurun_out/gpu_r6d.txt | head; exit $rc
