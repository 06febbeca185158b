#!/bin/bash
# round-4: shading-threshold sweep after the dedupe and the unrolled loop (C4, C2)
export TMPDIR=/tmp; mkdir -p gpurun_out
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats"
bash scripts/ab_env.sh <<AB
c4s48 RT_SHADE_MIN=48 $C4
c4s52 RT_SHADE_MIN=52 $C4
c4s56 RT_SHADE_MIN=56 $C4
c4s60 RT_SHADE_MIN=60 $C4
c4s62 RT_SHADE_MIN=62 $C4
c2s56 RT_SHADE_MIN=56 --no-stats
c2s60 RT_SHADE_MIN=60 --no-stats
c2s62 RT_SHADE_MIN=62 --no-stats
c4s56_b RT_SHADE_MIN=56 $C4
c4s60_b RT_SHADE_MIN=60 $C4
c2s56_b RT_SHADE_MIN=56 --no-stats
c2s60_b RT_SHADE_MIN=60 --no-stats
AB
