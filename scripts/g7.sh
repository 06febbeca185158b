# round-4: GPU suite; same-box A/B (deferred validation, Markstein quotients, refill / shading
# thresholds); strong-scaling estimates (C2, C5 shares)
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats"
cat > /tmp/ab.txt <<AB
c5 $C5
c5nodefer RT_HIP_LIB=build/ab/libnodefer.so $C5
c5ms RT_HIP_LIB=build/ab/libms.so $C5
c5ms2 RT_HIP_LIB=build/ab/libms2.so $C5
c5r8 RT_HIP_LIB=build/ab/librefill8.so $C5
c5r24 RT_HIP_LIB=build/ab/librefill24.so $C5
c5r32 RT_HIP_LIB=build/ab/librefill32.so $C5
c5ecull RT_HIP_LIB=build/ab/libecull.so $C5
c5_b $C5
c3 $C3
c3ecull RT_HIP_LIB=build/ab/libecull.so $C3
c3ms RT_HIP_LIB=build/ab/libms.so $C3
c3ms2 RT_HIP_LIB=build/ab/libms2.so $C3
c3r8 RT_HIP_LIB=build/ab/librefill8.so $C3
c3r32 RT_HIP_LIB=build/ab/librefill32.so $C3
c2 --no-stats
c2ms RT_HIP_LIB=build/ab/libms.so --no-stats
c4 $C4
c4ms RT_HIP_LIB=build/ab/libms.so $C4
c4s40 RT_SHADE_MIN=40 $C4
c4s56 RT_SHADE_MIN=56 $C4
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
timeout -k 10 300 python -u scripts/diag_scale.py > gpurun_out/scale_c2.log 2>&1; echo scale c2 rc=$?; cat gpurun_out/scale_c2.log
VERBOSE=1 timeout -k 10 400 python -u scripts/diag_scale.py final 3840 2159 100 1 > gpurun_out/scale_c5.log 2>&1; echo scale c5 rc=$?; grep "^N=" gpurun_out/scale_c5.log
