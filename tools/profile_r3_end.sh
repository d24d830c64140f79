# End-of-round-3 profile of the headline bench (GPU box): rocprofv3 kernel
# statistics, then one PMC pass of the wave kernel's instruction mix
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/bench.py --steps 20 --warmup 5 --no-extras"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_end -o run --output-format csv -- $B > $R/gpurun_out/prof_end.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d $R/gpurun_out/pmc_end -o run --output-format csv -- $B > $R/gpurun_out/pmc_end.log 2>&1
