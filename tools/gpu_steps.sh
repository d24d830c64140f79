#!/bin/bash
# Run GPU steps one after another under their own time limits; a step that
# ends with a test failure (exit 1) lets the next one run, anything else
# (timeout 124/137, abort 134, segfault 139, ...) ends the script there.
#   tools/gpu_steps.sh "<name>|<seconds>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "=== $name ($secs s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc $(( $(date +%s) - start )) s"
    tail -5 "gpurun_out/$name.log"
    # a device fault inside a test (pytest exit 1) ends the script as well
    if grep -q -E "illegal memory access|Memory access fault|HIP error|hipError|GPU fault" "gpurun_out/$name.log"; then
        echo "=== stopping after $name: device fault in the log"
        exit 3
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "=== stopping after $name (rc=$rc)"
        exit $rc
    fi
done
