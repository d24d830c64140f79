# rocprofv3 kernel statistics of a short bench.py run (30 qubits, fp64,
# wave-tile engine) plus PMC counters of the wave kernel (tools/pmc_wave.sh);
# run on the GPU box, results under gpurun_out/
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 &&
bash $R/tools/pmc_wave.sh
