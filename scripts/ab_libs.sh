#!/bin/bash
# Same-box A/B of librt_hip.so builds (scripts/build_ab.sh) on one bench workload: every build REPS
# times (default 2), interleaved, one bench.py line each.
#   bash scripts/ab_libs.sh c4 "--scene door --width 1920 --height 1079 --spp 16 --nfb 16" \
#        base=build/ab/libbase.so new=raytracing_gpu_amd/librt_hip.so
set -u
mkdir -p gpurun_out
tag=$1; args=$2; shift 2
for rep in $(seq 1 ${REPS:-2}); do
  for pair in "$@"; do
    name=${pair%%=*}; lib=${pair#*=}
    log=gpurun_out/ab_${tag}_${name}_$rep.log
    RT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py $args --steps ${STEPS_AB:-5} --warmup 2 --warm-steps 2 \
      --no-cpu-baseline --no-stats ${AB_ARGS:-} > $log 2>&1
    rc=$?
    echo "$tag $name #$rep rc=$rc $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"warm_kernel_ms": [0-9.]*' $log | tr '\n' ' ')"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
