#!/bin/bash
# Same-box A/B of the 17-qubit density-matrix channel workload (bench.py's
# density17 extra) under planner knobs; one process per variant (each
# allocates the 256 GiB matrix afresh):
#   bash tools/density_knobs_ab.sh "name|VAR=x VAR2=y" ...
for spec in "$@"; do
    IFS='|' read name envs <<< "$spec"
    out=$( (for kv in $envs; do export "$kv"; done
            timeout -k 10 200 python -c "
import quest_amd as qa
from quest_amd.utils.bench_workloads import run_density17
res = {}
run_density17(qa.Env(), res)
") 2>&1) || { echo "$name FAILED: $out" | tail -3; exit 1; }
    echo "$name $(echo "$out" | grep '^density17')"
done
