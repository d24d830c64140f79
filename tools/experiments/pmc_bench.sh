# PMC counters of the wave-tile kernel on the headline bench (30 qubits, 3
# layers), one rocprofv3 pass per counter group (run on the GPU box:
# bash tools/experiments/pmc_bench.sh); summaries -> gpurun_out/pmcb_*
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 3 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $R/gpurun_out/pmcb_a -o run --output-format csv -- python3 $B > $R/gpurun_out/pmcb_a.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS -d $R/gpurun_out/pmcb_b -o run --output-format csv -- python3 $B > $R/gpurun_out/pmcb_b.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $R/gpurun_out/pmcb_c -o run --output-format csv -- python3 $B > $R/gpurun_out/pmcb_c.log 2>&1
