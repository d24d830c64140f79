#!/bin/bash
# GPU box: per-pass times of the headline circuit in three builds -- full,
# compute only (tools/gen_wave_asm.py --nomem library in quest_amd/lib/var/
# nomem.so) and memory only (QUEST_WAVE_NOOPS=1) -- each joined with the pass
# trace (tools/pass_profile.py); then tools/pass_overlap.py compares them.
# VARIANTS="noops": only some of the three; TAG=x: output under gpurun_out/po<seed>x.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-full nomem noops}; do
  mkdir -p $R/gpurun_out/po${SEED:-}${TAG:-}/$v
  unset QUEST_LIB QUEST_WAVE_NOOPS
  [ $v = nomem ] && export QUEST_LIB=${NOMEM_LIB:-$R/quest_amd/lib/var/nomem.so}
  [ $v = noops ] && export QUEST_WAVE_NOOPS=1
  QUEST_TRACE=$R/gpurun_out/po${SEED:-}${TAG:-}/$v/trace.jsonl timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
      -d $R/gpurun_out/po${SEED:-}${TAG:-}/$v -o run -- python3 $R/tools/pass_profile.py run --qubits ${QUBITS:-30} --layers ${LAYERS:-25} --seed ${SEED:-7} \
      > $R/gpurun_out/po${SEED:-}${TAG:-}/$v/run.log 2>&1 || exit $?
  python3 $R/tools/pass_profile.py join $R/gpurun_out/po${SEED:-}${TAG:-}/$v > $R/gpurun_out/po${SEED:-}${TAG:-}/$v/passes.txt 2>&1 || exit $?
done
