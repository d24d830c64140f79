#!/bin/bash
# Next-tile prefetch variants of the wave kernel (ab_libs/<v>/libQuEST_hip_f64.so,
# built with make WAVE_PFA=.. WAVE_PFL=..): GPU correctness of each (looping grids
# bit-equal to one tile per workgroup, every gate kind vs the oracle), then the
# headline bench interleaved.  VARIANTS="pf55 pf275"; ROUNDS=2.
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in default ${VARIANTS:-pf55 pf275}; do
  if [ $v = default ]; then unset QUEST_LIB; else export QUEST_LIB=$R/ab_libs/$v/libQuEST_hip_f64.so; fi
  timeout -k 10 400 python -u -m pytest tests/test_wave.py -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "looping_grids or (every_gate_kind_gpu and not fp32)" > gpurun_out/pf_check_$v.log 2>&1 \
      || { echo "check $v failed"; tail -30 gpurun_out/pf_check_$v.log; exit 1; }
  echo "check $v: $(tail -1 gpurun_out/pf_check_$v.log)"
done
unset QUEST_LIB
ARGS=(default)
for v in ${VARIANTS:-pf55 pf275}; do ARGS+=($R/ab_libs/$v/libQuEST_hip_f64.so); done
bash tools/ab_libs_multi.sh ${ROUNDS:-2} "${ARGS[@]}"
