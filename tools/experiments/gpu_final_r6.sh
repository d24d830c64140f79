#!/bin/bash
# End of round 6: smoke() as the driver runs it, then the whole GPU suite with durations.
set -o pipefail
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6.txt 2>&1 || { cat gpurun_out/smoke_r6.txt; exit 1; }
tail -1 gpurun_out/smoke_r6.txt
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/gpu_suite_r6.txt 2>&1
rc=$?
tail -20 gpurun_out/gpu_suite_r6.txt
exit $rc
