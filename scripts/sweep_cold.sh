#!/bin/bash
# Cold-draw sweep of one tuning variable ($VAR, values $VALS) with diag_scale.py's cold columns,
# C2 10 x 10 and 1 x 100.
mkdir -p gpurun_out
VAR=${VAR:-RT_HOT_SEGS_PER_SAMPLE}; VALS=${VALS:-0 2 4 8}
o=gpurun_out/sweep_cold.log; : > $o
one() { echo "== $VAR=$1 ${*:2}" >> $o; env $VAR=$1 timeout -k 10 300 python scripts/diag_scale.py "${@:2}" 2>/dev/null | grep "N=" >> $o || exit 1; }
for v in $VALS; do one $v || exit 1; done
for v in $VALS; do one $v big1 1200 800 100 1 || exit 1; done
cat $o
