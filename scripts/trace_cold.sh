#!/bin/bash
# rocprofv3 kernel trace of one-shot draws (bench.py's timed leg only: no warm leg, no stats pass):
# the probe twin, the schedule kernels and the render kernel of each draw, with their gaps.
#   NAME=c2 ARGS="" bash scripts/trace_cold.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NAME=${NAME:-c2}
timeout -k 10 ${STEP_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d gpurun_out/cold_${NAME} -o run --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --warm-steps 0 --no-cpu-baseline --no-stats ${ARGS:-} > gpurun_out/cold_${NAME}.log 2>&1
rc=$?
echo "cold_${NAME} rc=$rc"
[ $rc -eq 0 ] || exit $rc
python scripts/trace_gaps.py gpurun_out/cold_${NAME} > gpurun_out/cold_${NAME}_gaps.txt && tail -40 gpurun_out/cold_${NAME}_gaps.txt
