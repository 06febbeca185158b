#!/bin/bash
# round-4: C3's variant at 5 waves/SIMD (96 VGPRs, 16 spilled) vs 4 (108, none): parity of the wpe5
# library on the C3 tests, then same-box A/B
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_HIP_LIB=build/ab/libwpe5.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "cornell_smoke" > gpurun_out/t_wpe5.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_wpe5.log | tail -5; echo wpe5 rc=$rc; [ $rc = 0 ] || exit $rc
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
bash scripts/ab_env.sh <<AB
c3 $C3
c3w5 RT_HIP_LIB=build/ab/libwpe5.so $C3
c3_b $C3
c3w5_b RT_HIP_LIB=build/ab/libwpe5.so $C3
AB
