R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for seed in 7 1 2 3 4; do
    for v in default v5w2nolp; do
      if [ "$v" = default ]; then unset QUEST_LIB QUEST_WAVE_LOW_PERM; else export QUEST_LIB=$R/ab_libs/v5w2/libQuEST_hip_f64.so QUEST_WAVE_LOW_PERM=0; fi
      timeout -k 10 120 python bench.py --no-extras --steps 20 --warmup 5 --seed $seed > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('seed $seed $v', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
    done
  done
done
