#!/bin/bash
# Quick A/B of bench variants on the GPU box: each line = one bench invocation (args after the name).
mkdir -p gpurun_out
while read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $args > gpurun_out/ab_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -o "\"value\": [0-9.]*" gpurun_out/ab_$name.log) $(grep -o "\"kernel_avg_ms\": [0-9.]*" gpurun_out/ab_$name.log) $(grep -o "\"node_tests_per_segment\": [0-9.]*" gpurun_out/ab_$name.log) $(grep -o "\"fallbacks\": [0-9]*" gpurun_out/ab_$name.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
