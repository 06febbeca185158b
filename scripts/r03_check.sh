#!/bin/bash
# Round-3 GPU check: parity suite, smoke, default bench, C2 primary split (1 x 100) bench,
# in-process two-rank bench.  Stops at the first crash-like exit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd... (env assignments before `run` apply to the command)
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/summary.txt
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/summary.txt
  tail -3 "gpurun_out/$name.log"
  if crash $rc; then echo "CRASH in $name, stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests smoke bench b1x100}
for s in $STEPS; do
  case $s in
    tests) run tests 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 5 ;;
    b1x100) run b1x100 300 python bench.py --steps 5 --warmup 2 --nfb 1 --spp 100 --no-cpu-baseline ;;
    scale) run scale 300 python scripts/diag_scale.py ;;
    scale0) DIAG_PROBE=0 run scale0 300 python scripts/diag_scale.py ;;
    s1x100) run s1x100 300 python scripts/diag_scale.py big1 1200 800 100 1 ;;
    cold) run cold 400 python scripts/diag_cold.py ;;
    cold1x100) run cold1x100 400 python scripts/diag_cold.py big1 1200 800 100 1 ;;
    pace) run pace 300 python scripts/diag_pace.py ;;
    split) run split 400 python scripts/diag_split.py ;;
    splitb) run splitb 400 python scripts/diag_split.py 100 1 default 300 350 400 450 500 600 ;;
    split10) run split10 400 python scripts/diag_split.py 10 10 default 12 24 48 96 ;;
    b2host) run b2host 300 python bench.py --gpus 2 --gather host --steps 5 --warmup 2 ;;
  esac
done
