#!/bin/bash
# A/B of bench variants on the GPU box.  Each stdin line: name [ENV=value ...] [bench args ...].
mkdir -p gpurun_out
while read -r name rest; do
  [ -z "$name" ] && continue
  envs=(); args=()
  for w in $rest; do case $w in *=*) envs+=("$w");; *) args+=("$w");; esac; done
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-cpu-baseline "${args[@]}" > gpurun_out/ab_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -o "\"value\": [0-9.]*" gpurun_out/ab_$name.log) $(grep -o "\"kernel_avg_ms\": [0-9.]*" gpurun_out/ab_$name.log) $(grep -o "\"fallbacks\": [0-9]*" gpurun_out/ab_$name.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
