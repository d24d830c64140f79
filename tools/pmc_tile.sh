# rocprofv3 kernel trace + two PMC passes of the fused tile kernel on tools/tile_workload.py
# (run on the GPU box: bash tools/pmc_tile.sh; results under gpurun_out/pmc_*)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc_t -o run --output-format csv -- python3 $R/tools/tile_workload.py > $R/gpurun_out/pmc_t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc_a -o run --output-format csv -- python3 $R/tools/tile_workload.py > $R/gpurun_out/pmc_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES -d $R/gpurun_out/pmc_b -o run --output-format csv -- python3 $R/tools/tile_workload.py > $R/gpurun_out/pmc_b.log 2>&1
