#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.  Stops at the first
# crash-like exit (timeout, abort, segfault); a plain test failure does not stop the bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/summary.txt
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/summary.txt
  tail -5 "gpurun_out/$name.log"
  if crash $rc; then echo "CRASH in $name, stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests smoke bench prof}
for s in $STEPS; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 3 --warmup 1 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
  esac
done
