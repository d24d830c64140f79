#!/bin/bash
# Final distributed GPU checks on the default chain lengths: swap / fuzz / distributed tests and the torchrun dist bench tests.
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests/test_gpu.py tests/test_fuzz_dist.py tests/test_distributed.py tests/test_gpu_dist_bench.py -m gpu -x -v -s \
    --timeout 300 --timeout-method thread -k "ranges or overlapped or fuzz or ipc or rccl or torchrun" > gpurun_out/dist_final_r6.txt 2>&1
rc=$?
grep -E "per window|passed|failed|FAILED" gpurun_out/dist_final_r6.txt | tail -8
exit $rc
