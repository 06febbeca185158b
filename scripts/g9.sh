# round-4 A/B: render_kernel refill threshold (kRefill) and the deferred validation, C5 and C3
export TMPDIR=/tmp; mkdir -p gpurun_out
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
cat > /tmp/ab.txt <<AB
c5r16 $C5
c5r8 RT_HIP_LIB=build/ab/librefill8.so $C5
c5r4 RT_HIP_LIB=build/ab/librefill4.so $C5
c5r2 RT_HIP_LIB=build/ab/librefill2.so $C5
c5r1 RT_HIP_LIB=build/ab/librefill1.so $C5
c5r8nd RT_HIP_LIB=build/ab/libr8nodefer.so $C5
c3r16 $C3
c3r8 RT_HIP_LIB=build/ab/librefill8.so $C3
c3r4 RT_HIP_LIB=build/ab/librefill4.so $C3
c3r2 RT_HIP_LIB=build/ab/librefill2.so $C3
c3r1 RT_HIP_LIB=build/ab/librefill1.so $C3
c5r8_b RT_HIP_LIB=build/ab/librefill8.so $C5
c5r4_b RT_HIP_LIB=build/ab/librefill4.so $C5
c5r8nd_b RT_HIP_LIB=build/ab/libr8nodefer.so $C5
c3r8_b RT_HIP_LIB=build/ab/librefill8.so $C3
c3r4_b RT_HIP_LIB=build/ab/librefill4.so $C3
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
