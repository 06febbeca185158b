#!/bin/bash
# round-4: GPU suite with the deduplicated traversal trees, then same-box A/B: dedupe vs RT_NO_DEDUP
# (C4, C5), 2x-unrolled traversal loop (build/ab/libunroll2.so, built without dedupe) on C2 / C4
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; [ $rc = 0 ] || exit $rc
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16"
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4"
bash scripts/ab_env.sh <<AB
c4 $C4
c4nodedup RT_NO_DEDUP=1 $C4
c4u2 RT_HIP_LIB=build/ab/libunroll2.so $C4
c5 $C5
c5nodedup RT_NO_DEDUP=1 $C5
c2 
c2u2 RT_HIP_LIB=build/ab/libunroll2.so
c4_b $C4
c4nodedup_b RT_NO_DEDUP=1 $C4
c2_b 
c2u2_b RT_HIP_LIB=build/ab/libunroll2.so
AB
