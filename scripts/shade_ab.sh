#!/bin/bash
set -u
mkdir -p gpurun_out
for rep in 1 2; do for sm in ${SMS:-0 48 52 60}; do
  timeout -k 10 300 python -u bench.py --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --steps 5 --warmup 2 --cold-steps 1 --no-cpu-baseline --no-stats --opt shade_min=$sm > gpurun_out/sm_${sm}_$rep.log 2>&1 || exit $?
  echo "c4 shade_min=$sm #$rep $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/sm_${sm}_$rep.log | tr '\n' ' ')"
done; done
