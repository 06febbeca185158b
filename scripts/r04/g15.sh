#!/bin/bash
# round-4: GPU suite with two traversal steps per shading check, then C4 knobs after the dedupe
# (shading threshold, quantized LDS tree on/off) and C2/C5 bench lines
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; [ $rc = 0 ] || exit $rc
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats"
bash scripts/ab_env.sh <<AB
c2 --no-stats
c4 $C4
c4s40 RT_SHADE_MIN=40 $C4
c4s56 RT_SHADE_MIN=56 $C4
c4noq RT_NO_QLDS=1 $C4
c5 --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c2_b --no-stats
c4_b $C4
AB
