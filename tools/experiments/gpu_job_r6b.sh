#!/bin/bash
# round-6 swap ranges + IPC mapping cache + footprint: the distributed GPU tests
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_footprint_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
   -k "ranges or overlapped or rank_controlled or footprint or distributed_equivalence or ipc" > gpurun_out/gpu_r6b.txt 2>&1
rc=$?; tail -8 gpurun_out/gpu_r6b.txt; exit $rc
