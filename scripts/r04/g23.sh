#!/bin/bash
# round-4: C3's variant at 5 waves/SIMD (new default, no traversal stacks in LDS), and with its
# per-segment state parked in the LDS locker at 5 and 6 waves: C3 parity of each, then A/B
export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in "" build/ab/libpark5.so build/ab/libpark6.so; do
  RT_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "cornell" > gpurun_out/t_c3.log 2>&1; rc=$?
  echo "lib=${lib:-default} $(grep -E 'passed|failed' gpurun_out/t_c3.log | tail -1) rc=$rc"; [ $rc = 0 ] || exit $rc
done
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
bash scripts/ab_env.sh <<AB
c3 $C3
c3p5 RT_HIP_LIB=build/ab/libpark5.so $C3
c3p6 RT_HIP_LIB=build/ab/libpark6.so $C3
c3_b $C3
c3p5_b RT_HIP_LIB=build/ab/libpark5.so $C3
c3p6_b RT_HIP_LIB=build/ab/libpark6.so $C3
AB
