# HBM traffic of the unfused kernels (tools/experiments/direct_pmc.py, 28 qubits):
# FETCH_SIZE and WRITE_SIZE (KiB per dispatch) in separate rocprofv3 passes
# (one pass holds at most 4 TCC counters); run on the GPU box
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_direct_$c -o run --output-format csv -- python3 $R/tools/experiments/direct_pmc.py 28 > $R/gpurun_out/pmc_direct_$c.log 2>&1 || exit $?
done
