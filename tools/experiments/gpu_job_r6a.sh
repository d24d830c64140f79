set -o pipefail
N=6 bash tools/experiments/placement_r6.sh > gpurun_out/placement_r6c.txt 2>&1 || { echo placement failed; tail -20 gpurun_out/placement_r6c.txt; exit 1; }
cat gpurun_out/placement_r6c.txt
timeout -k 10 600 python -u -m pytest tests/test_fuzz_dist.py tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fuzz or rank_controlled or overlapped" > gpurun_out/gpu_fuzz.txt 2>&1; rc=$?
tail -15 gpurun_out/gpu_fuzz.txt; exit $rc
