#!/bin/bash
# round-4: traversal steps per shading check: 2 (default) vs 3 / 4 (build/ab/libunroll{3,4}.so), C2 and C4
export TMPDIR=/tmp; mkdir -p gpurun_out
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats"
bash scripts/ab_env.sh <<AB
c2 --no-stats
c2u3 RT_HIP_LIB=build/ab/libunroll3.so --no-stats
c2u4 RT_HIP_LIB=build/ab/libunroll4.so --no-stats
c4 $C4
c4u3 RT_SHADE_MIN=56 RT_HIP_LIB=build/ab/libunroll3.so $C4
c4u4 RT_SHADE_MIN=56 RT_HIP_LIB=build/ab/libunroll4.so $C4
c2_b --no-stats
c2u3_b RT_HIP_LIB=build/ab/libunroll3.so --no-stats
c2u4_b RT_HIP_LIB=build/ab/libunroll4.so --no-stats
AB
