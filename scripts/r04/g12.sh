#!/bin/bash
# round-4: parity of the merged list-world search, then same-box A/B (merge vs RT_NO_MERGE) on C5/C3
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_shares_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_shares.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_shares.log | tail -20; echo shares rc=$rc; [ $rc = 0 ] || exit $rc
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
bash scripts/ab_env.sh <<AB
c5 $C5
c5nomerge RT_NO_MERGE=1 $C5
c5_b $C5
c5nomerge_b RT_NO_MERGE=1 $C5
c3 $C3
c3nomerge RT_NO_MERGE=1 $C3
AB
