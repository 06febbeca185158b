#!/bin/bash
# bench.py lines of one workload under several context options (--opt KEY=VALUE; several options
# of one run joined by commas), REPS rounds:
#   bash scripts/opt_sweep.sh c2 "" shade_min=0 shade_min=56 probe_schedule=4,probe_max_items_per_lane=1000 ...
set -u
mkdir -p gpurun_out
tag=$1; args=$2; shift 2
for rep in $(seq 1 ${REPS:-2}); do for o in "$@"; do
  timeout -k 10 300 python -u bench.py $args --steps ${STEPS_AB:-5} --warmup 2 --warm-steps 2 --no-cpu-baseline --no-stats $(echo ",$o" | sed 's/,/ --opt /g') > gpurun_out/sw_${tag}_${o//[=.,]/_}_$rep.log 2>&1 || exit $?
  echo "$tag $o #$rep $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"warm_kernel_ms": [0-9.]*' gpurun_out/sw_${tag}_${o//[=.,]/_}_$rep.log | tr '\n' ' ')"
done; done
