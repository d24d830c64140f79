# rocprofv3 kernel stats + PMC passes of the wave-tile kernel (tile mode 3)
# on the layered circuit (run on the GPU box: bash tools/pmc_wave.sh)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
W="python3 $R/tools/wave_check.py --skip-check --modes 3 --qubits 28 --layers 4 --rounds 1"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmcw_t -o run --output-format csv -- $W > $R/gpurun_out/pmcw_t.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $R/gpurun_out/pmcw_a -o run --output-format csv -- $W > $R/gpurun_out/pmcw_a.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS -d $R/gpurun_out/pmcw_b -o run --output-format csv -- $W > $R/gpurun_out/pmcw_b.log 2>&1
