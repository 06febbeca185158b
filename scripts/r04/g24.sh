#!/bin/bash
# round-4: world_search's visiting order of C5's list entries (RT_MERGE_ORDER): parity of the merged
# search under a permuted order, then same-box A/B of several orders
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_MERGE_ORDER=prims timeout -k 10 600 python -u -m pytest tests/test_shares_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -k "merged or final" > gpurun_out/t_order.log 2>&1; rc=$?
echo "order=prims $(grep -E 'passed|failed' gpurun_out/t_order.log | tail -1) rc=$rc"; [ $rc = 0 ] || exit $rc
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
bash scripts/ab_env.sh <<AB
c5 $C5
c5prims RT_MERGE_ORDER=prims $C5
c5pdi RT_MERGE_ORDER=1,2,3,4,5,8,9,11,10,0,6,7 $C5
c5bvh RT_MERGE_ORDER=0,11,10,1,2,3,4,5,8,9,6,7 $C5
c5pgd RT_MERGE_ORDER=1,2,3,4,5,8,9,0,11,10,6,7 $C5
c5_b $C5
c5prims_b RT_MERGE_ORDER=prims $C5
AB
