# Address-translation counters of the bare wave pass (QUEST_WAVE_NOOPS=1) for
# a contiguous tile vs a tile of the 9 highest qubits (tools/experiments/tile_layout_probe.py)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export QUEST_WAVE_NOOPS=1
for set in contiguous "0-3 + top"; do
  tag=$(echo $set | tr -c 'a-z0-9\n' '_')
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $R/gpurun_out/pmct_$tag -o run --output-format csv -- python3 $R/tools/experiments/tile_layout_probe.py --only "$set" --reps 3 > $R/gpurun_out/pmct_$tag.log 2>&1 || exit $?
done
