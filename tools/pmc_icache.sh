# instruction-cache counters of the wave-tile kernel (one PMC pass; run on the GPU box)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
W="python3 $R/tools/wave_check.py --skip-check --modes 3 --qubits 28 --layers 4 --rounds 1"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $R/gpurun_out/pmci -o run --output-format csv -- $W > $R/gpurun_out/pmci.log 2>&1
