#!/bin/bash
# Split-threshold sweep per share (diag_split.py), C2 1 x 100 and 10 x 10; extra env from $SWEEP_ENV (e.g. RT_HIP_LIB=build/ab/libX.so).
mkdir -p gpurun_out
o=gpurun_out/sweep.log; : > $o
one() { echo "N=$1 ${SWEEP_ENV:-}" >> $o; env ${SWEEP_ENV:-} DIAG_N=$1 timeout -k 10 300 python scripts/diag_split.py "${@:2}" 2>/dev/null | grep warm >> $o || exit 1; }
one 1 100 1 default 200 300 400 &&
one 2 100 1 default 100 200 300 400 &&
one 4 100 1 default 50 100 150 200 250 &&
one 8 100 1 default 50 70 85 100 120 &&
one 1 10 10 default 24 32 48 64 &&
one 2 10 10 default 24 32 48 64 &&
one 4 10 10 default 24 32 48 64 &&
one 8 10 10 default 16 24 32 40 48
cat $o
