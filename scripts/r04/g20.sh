#!/bin/bash
# round-4: C4's quantized LDS tree sized from the deduplicated tree's own record count: GPU suite,
# then same-box A/B with and without it (RT_NO_QLDS=1)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; [ $rc = 0 ] || exit $rc
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16"
bash scripts/ab_env.sh <<AB
c4 $C4
c4noq RT_NO_QLDS=1 $C4
c4s48 RT_SHADE_MIN=48 $C4
c4s60 RT_SHADE_MIN=60 $C4
c4_b $C4
c4noq_b RT_NO_QLDS=1 $C4
AB
