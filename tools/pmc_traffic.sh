# HBM traffic counters of a known-byte copy, the unfused kernels and a wave
# pass (tools/pmc_traffic.py), one rocprofv3 pass per counter group (a pass
# holds at most 4 TCC counters; FETCH_SIZE takes 3, WRITE_SIZE 2).  Run on
# the GPU box; results under gpurun_out/pmc_traffic_*.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc_traffic_$i -o run --output-format csv -- python3 $R/tools/pmc_traffic.py 28 > $R/gpurun_out/pmc_traffic_$i.log 2>&1 || exit $?
done
