#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; a step that ends in
# a fault-like way (timeout 124/137, abort 134, segfault 139, or a signal)
# stops the whole sequence, an ordinary failure (e.g. pytest exit 1) does not.
#
# usage: tools/gpu_steps.sh "<seconds>|<name>|<command>" ...
# output of each step -> gpurun_out/<name>.log ; summary -> gpurun_out/steps.txt
mkdir -p gpurun_out
: > gpurun_out/steps.txt
for spec in "$@"; do
    secs="${spec%%|*}"
    rest="${spec#*|}"
    name="${rest%%|*}"
    cmd="${rest#*|}"
    echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/steps.txt
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    end=$(date +%s)
    echo "=== $name rc=$rc time=$((end - start))s" | tee -a gpurun_out/steps.txt
    tail -5 "gpurun_out/$name.log"
    case $rc in
        0|1|2|3|4|5) ;;
        *) echo "stopping after fault-like exit $rc" | tee -a gpurun_out/steps.txt; exit $rc ;;
    esac
done
exit 0
