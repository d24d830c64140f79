# Round-2 end profile: rocprofv3 kernel statistics of the driver-config bench
# (the timed window + the unfused-gate probe, now on the direct kernels) and
# the full benchmark suite.  Run on the GPU box; results under gpurun_out/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_end -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras > $R/gpurun_out/prof_end.log 2>&1 || exit $?
cd $R
timeout -k 10 600 python3 -u tools/bench_suite.py --out gpurun_out/bench_suite_end.json > gpurun_out/bench_suite_end.log 2>&1
