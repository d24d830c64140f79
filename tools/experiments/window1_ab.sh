for r in 1 2; do for v in base new; do
  if [ $v = base ]; then export QUEST_LIB=$PWD/ab_libs/base/libQuEST_hip_f64.so; else unset QUEST_LIB; fi
  timeout -k 10 200 python bench.py --extras window1 > gpurun_out/w1.json 2> gpurun_out/w1.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/w1.json') if l.startswith('{')][0]); c=d['config']; print('$v', round(d['value']*1e3,4), c['seed7_s_per_gate']*1e3, c['window1_s_per_gate']*1e3)"
done; done
