#!/bin/bash
# round-4: C4's quantized-tree variant with materials, textures and images staged in LDS
# (build/ab/libtables.so: this change on the final round-4 source, committed after the run): GPU suite on
# that library, then same-box A/B against the tree's kernels
export TMPDIR=/tmp; mkdir -p gpurun_out
RT_HIP_LIB=build/ab/libtables.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_tables.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_tables.log | tail -20; echo tables rc=$rc; [ $rc = 0 ] || exit $rc
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats"
bash scripts/ab_env.sh <<AB
c4 $C4
c4tables RT_HIP_LIB=build/ab/libtables.so $C4
c4_b $C4
c4tables_b RT_HIP_LIB=build/ab/libtables.so $C4
AB
