#!/bin/bash
# round-4: scalar loads of the list entries in world_search (C5's merged search) and of the step
# kernel's trailing primitives (C4's ground sphere): GPU suite, then same-box A/B against
# build/ab/libbase.so (the kernels before any scalar loads)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; [ $rc = 0 ] || exit $rc
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats"
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats"
bash scripts/ab_env.sh <<AB
c5 $C5
c5base RT_HIP_LIB=build/ab/libbase.so $C5
c4 $C4
c4base RT_HIP_LIB=build/ab/libbase.so $C4
c2 --no-stats
c2base RT_HIP_LIB=build/ab/libbase.so --no-stats
c5_b $C5
c5base_b RT_HIP_LIB=build/ab/libbase.so $C5
c4_b $C4
c4base_b RT_HIP_LIB=build/ab/libbase.so $C4
c2_b --no-stats
c2base_b RT_HIP_LIB=build/ab/libbase.so --no-stats
AB
