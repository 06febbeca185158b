#!/bin/bash
# round-4: GPU suite with scalar (constant address space) scene loads in the list-world variants
# without BVHs (C3), then same-box A/B against the previous kernels (build/ab/libbase.so)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; [ $rc = 0 ] || exit $rc
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
bash scripts/ab_env.sh <<AB
c3 $C3
c3base RT_HIP_LIB=build/ab/libbase.so $C3
c3_b $C3
c3base_b RT_HIP_LIB=build/ab/libbase.so $C3
c2 --no-stats
c2base RT_HIP_LIB=build/ab/libbase.so --no-stats
AB
