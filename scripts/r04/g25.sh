#!/bin/bash
# round-4: default world_search visiting order (primitives, then BVH / instance entries nearest the
# camera first): GPU suite, then same-box A/B against list order and the explicit C5 permutation
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; [ $rc = 0 ] || exit $rc
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
bash scripts/ab_env.sh <<AB
c5 $C5
c5list RT_MERGE_ORDER=list $C5
c5pgd RT_MERGE_ORDER=1,2,3,4,5,8,9,0,11,10,6,7 $C5
c5_b $C5
c5list_b RT_MERGE_ORDER=list $C5
AB
