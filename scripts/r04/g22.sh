#!/bin/bash
# round-4: C3's variant at 4 / 5 / 6 waves per SIMD (108 VGPRs / 96 with 16 spilled / 80 with 46 spilled)
export TMPDIR=/tmp; mkdir -p gpurun_out
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
bash scripts/ab_env.sh <<AB
c3 $C3
c3w5 RT_HIP_LIB=build/ab/libwpe5.so $C3
c3w6 RT_HIP_LIB=build/ab/libwpe6.so $C3
c3w6_b RT_HIP_LIB=build/ab/libwpe6.so $C3
c3w5_b RT_HIP_LIB=build/ab/libwpe5.so $C3
AB
