#!/bin/bash
# Program uploads through progUploadKernel (default) vs hipMemcpyAsync
# (QUEST_UPLOAD_KERNEL=0): fused_sweep rows, kernel gaps of 26-qubit windows.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_wave.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > $R/gpurun_out/upk_tests.txt 2>&1 || { tail -20 $R/gpurun_out/upk_tests.txt; exit 1; }
tail -2 $R/gpurun_out/upk_tests.txt
for rep in 1 2; do
  for e in 1 0; do
    QUEST_UPLOAD_KERNEL=$e timeout -k 10 200 python3 tools/experiments/sweep_ab.py --sizes 22 24 26 28 30 --tag "upload_kernel=$e" \
      >> $R/gpurun_out/upload_kernel_ab.txt 2> $R/gpurun_out/upload_kernel_ab.err || exit $?
    tail -1 $R/gpurun_out/upload_kernel_ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
QUEST_TRACE=$R/gpurun_out/wtk26.trace timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/wt_prof_upk -o run --output-format csv -- \
    python3 $R/tools/experiments/window_timeline.py --qubits 26 > $R/gpurun_out/wtk26.txt 2>&1 || exit $?
grep seed $R/gpurun_out/wtk26.txt
cd $R
for e in 1 0; do
  QUEST_UPLOAD_KERNEL=$e timeout -k 10 240 python bench.py --no-extras > gpurun_out/upk_bench.json 2>> gpurun_out/upload_kernel_ab.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/upk_bench.json')); print('bench upload_kernel=$e', '%.5g'%(d['value']*1e3), 'ms/gate', d['config']['passes'], [round(s['s_per_gate']*1e3,4) for s in d['config']['seeds']])" | tee -a gpurun_out/upload_kernel_ab.txt
done
