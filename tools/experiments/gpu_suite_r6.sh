#!/bin/bash
# The whole GPU suite (one pytest process, a line per test into gpurun_out/).
set -o pipefail
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite_r6.txt 2>&1
rc=$?
tail -5 gpurun_out/gpu_suite_r6.txt
exit $rc
