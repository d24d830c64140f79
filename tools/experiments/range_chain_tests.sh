#!/bin/bash
# GPU box: the swap-overlap tests after range-major chains of post-swap passes (QUEST_SWAP_RANGES_FIRST passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_fuzz_dist.py tests/test_distributed.py -m gpu -x -v -s \
    --timeout 300 --timeout-method thread -k "ranges or overlapped or fuzz or ipc or rccl" > gpurun_out/range_chain_tests.txt 2>&1
rc=$?
grep -E "per window|passed|failed|PASSED|FAILED" gpurun_out/range_chain_tests.txt | tail -40
exit $rc
