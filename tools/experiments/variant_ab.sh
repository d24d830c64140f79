# Wave-kernel build variants (ab_libs/<name>/libQuEST_hip_f64.so): a GPU
# correctness check of each, then the headline bench interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  [ "$v" = default ] && continue
  QUEST_LIB=$R/ab_libs/$v/libQuEST_hip_f64.so timeout -k 10 150 python -u -m pytest tests/test_wave.py -m gpu -x -q -k "every_gate_kind_gpu and not fp32" > gpurun_out/variant_check_$v.log 2>&1 || { echo "check $v failed"; tail -20 gpurun_out/variant_check_$v.log; exit 1; }
  echo "check $v ok"
done
ARGS=()
for v in "$@"; do if [ "$v" = default ]; then ARGS+=(default); else ARGS+=($R/ab_libs/$v/libQuEST_hip_f64.so); fi; done
bash tools/ab_libs_multi.sh 3 "${ARGS[@]}"
