#!/bin/bash
# round-4: C3's variant with materials and textures staged in LDS after its locker
# (build/ab/libc3tables.so: this change on the final source, committed after the run): GPU suite on that
# library, then same-box A/B against the tree's kernels
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_HIP_LIB=build/ab/libc3tables.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_c3tables.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_c3tables.log | tail -20; echo c3tables rc=$rc; [ $rc = 0 ] || exit $rc
C3="--scene cornell_smoke --width 800 --height 800 --no-stats"
bash scripts/ab_env.sh <<AB
c3 $C3
c3tables RT_HIP_LIB=build/ab/libc3tables.so $C3
c3_b $C3
c3tables_b RT_HIP_LIB=build/ab/libc3tables.so $C3
AB
