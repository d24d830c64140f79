# fp32 wave-tile shape variant (ab_libs/f32v/libQuEST_hip_f32.so) against the
# in-tree fp32 library: GPU check of every gate kind, then the headline bench
# in fp32 over circuit seeds, interleaved
R=$GRAFT_REPO_ROOT
export QUEST_PREC=1
QUEST_LIB=$R/ab_libs/f32v/libQuEST_hip_f32.so timeout -k 10 150 python -u -m pytest tests/test_wave.py -m gpu -x -q -k "fp32_wave_kernel_every_gate_kind_gpu" > gpurun_out/f32v_check.log 2>&1 || { echo "check failed"; tail -20 gpurun_out/f32v_check.log; exit 1; }
echo "check ok"
for round in 1 2; do
  for seed in 7 1 2 3; do
    for v in default f32v; do
      if [ "$v" = default ]; then unset QUEST_LIB; else export QUEST_LIB=$R/ab_libs/f32v/libQuEST_hip_f32.so; fi
      timeout -k 10 120 python bench.py --no-extras --steps 20 --warmup 5 --seed $seed > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('seed $seed $v', d['dtype'], round(d['value']*1e3, 4), 'ms/gate', d['config']['passes'], 'passes')"
    done
  done
done
