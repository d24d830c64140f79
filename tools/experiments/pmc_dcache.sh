# Scalar data cache behaviour of the wave-tile kernel on the headline bench
# (op records are read with s_load): one rocprofv3 PMC pass.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 3 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM -d $R/gpurun_out/pmcd -o run --output-format csv -- python3 $B > $R/gpurun_out/pmcd.log 2>&1
