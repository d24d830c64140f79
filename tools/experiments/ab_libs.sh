# A/B the headline bench between the in-tree library and another build of it
# on the same box: bash tools/experiments/ab_libs.sh <other.so> [rounds]
OTHER=$1
N=${2:-2}
for r in $(seq $N); do
  for v in new old; do
    if [ $v = old ]; then export QUEST_LIB=$OTHER; else unset QUEST_LIB; fi
    timeout -k 10 120 python bench.py > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
  done
done
