#!/bin/bash
# Cold-draw priority threshold sweep (RT_COLD_LONG_SEGS) with diag_scale.py's cold columns.
mkdir -p gpurun_out
o=gpurun_out/sweep_cold.log; : > $o
one() { echo "== RT_COLD_LONG_SEGS=$1 ${*:2}" >> $o; RT_COLD_LONG_SEGS=$1 timeout -k 10 300 python scripts/diag_scale.py "${@:2}" 2>/dev/null | grep "N=" >> $o || exit 1; }
one 0 && one 20 && one 40 && one 80 &&
one 0 big1 1200 800 100 1 && one 200 big1 1200 800 100 1 && one 400 big1 1200 800 100 1 && one 800 big1 1200 800 100 1
cat $o
