# A/B the headline bench between two environment settings on the same box:
# bash tools/experiments/ab_env.sh "VAR=a" "VAR=b" [rounds]
A=$1; B=$2; N=${3:-2}
for r in $(seq $N); do
  for v in "$A" "$B"; do
    env $v timeout -k 10 120 python bench.py > gpurun_out/ab_env.json 2> gpurun_out/ab_env.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_env.json')); print('$v', round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
  done
done
