# Headline bench of wave-kernel build variants (ab_libs/<name>) over circuit
# seeds, interleaved: bash tools/experiments/variant_seeds_ab.sh "7 1 2" default v5w2 ...
SEEDS=$1; shift
R=$GRAFT_REPO_ROOT
for round in 1 2; do
  for seed in $SEEDS; do
    for v in "$@"; do
      if [ "$v" = default ]; then unset QUEST_LIB; else export QUEST_LIB=$R/ab_libs/$v/libQuEST_hip_f64.so; fi
      timeout -k 10 120 python bench.py --no-extras --steps 20 --warmup 5 --seed $seed > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('seed $seed $v', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes', '%.1e' % d['config']['norm_error'])"
    done
  done
done
