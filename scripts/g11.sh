#!/bin/bash
# round-4: GPU suite on the merged list-world search (render_kernel, C5), then same-box A/B against
# the committed kernels (build/ab/libbase.so) and RT_NO_MERGE
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
cat > /tmp/ab.txt <<AB
c5 $C5
c5base RT_HIP_LIB=build/ab/libbase.so $C5
c5m1 RT_HIP_LIB=build/ab/libmerge1.so $C5
c5nomerge RT_NO_MERGE=1 $C5
c5_b $C5
c5base_b RT_HIP_LIB=build/ab/libbase.so $C5
c5m1_b RT_HIP_LIB=build/ab/libmerge1.so $C5
c3 $C3
c3base RT_HIP_LIB=build/ab/libbase.so $C3
c2 --no-stats
c2u2 RT_HIP_LIB=build/ab/libunroll2.so --no-stats
c2_b --no-stats
c2u2_b RT_HIP_LIB=build/ab/libunroll2.so --no-stats
c4 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
c4u2 RT_HIP_LIB=build/ab/libunroll2.so --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
