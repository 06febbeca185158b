#!/bin/bash
# bench cold legs by probe grid step
set -u
mkdir -p gpurun_out
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16"
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4"
for cfg in c2 c5 c4; do
  case $cfg in c2) args="";; c4) args=$C4;; c5) args=$C5;; esac
  for o in 4 2 1 0; do
    timeout -k 10 300 python -u bench.py $args --steps 3 --warmup 2 --cold-steps 3 --no-cpu-baseline --no-stats --opt probe_schedule=$o > gpurun_out/cold_${cfg}_$o.log 2>&1 || exit $?
    echo "$cfg probe=$o $(grep -o '"cold_kernel_ms": [0-9.]*\|"kernel_ms": [0-9.]*\|"cold_schedule_bits": \[[0-9, ]*\]' gpurun_out/cold_${cfg}_$o.log | tr '\n' ' ')"
  done
done
