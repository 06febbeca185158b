#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py exactly as the driver runs it (default arguments unless
# ARGS is set): the summary whose render-kernel average the bench line's kernel_ms is checked against.
#   NAME=c2 bash scripts/trace_bench.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NAME=${NAME:-c2}
timeout -k 10 ${STEP_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d gpurun_out/bench_trace_${NAME} -o run --output-format csv -- \
  python bench.py ${ARGS:-} > gpurun_out/bench_trace_${NAME}.log 2>&1
rc=$?
echo "bench_trace_${NAME} rc=$rc"
[ $rc -eq 0 ] || exit $rc
grep -h "render\|init_states\|resolve" gpurun_out/bench_trace_${NAME}/run_kernel_stats.csv
