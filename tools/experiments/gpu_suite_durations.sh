#!/bin/bash
# The whole GPU suite with per-test durations (one pytest process).
set -o pipefail
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=40 > gpurun_out/gpu_suite_durations.txt 2>&1
rc=$?
tail -50 gpurun_out/gpu_suite_durations.txt
exit $rc
