# Kernel statistics of bench.py with the current wave kernel, then the
# address-translation counters of the bench with the XCD/CU tile map on and
# off (QUEST_WAVE_TILE_MAP).  Run on the GPU box: bash tools/experiments/pmc_tilemap.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_bench.log 2>&1 || exit $?
for m in 1 0; do
  export QUEST_WAVE_TILE_MAP=$m
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $R/gpurun_out/pmcm_$m -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/pmcm_$m.log 2>&1 || exit $?
done
