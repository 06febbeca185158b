#!/bin/bash
# Round-3 evidence runs: default bench line (C2, roofline from profiles/r03, CPU baseline), C2's
# primary 1 x 100 split, the in-process two-rank driver, and C5 at its configured 10 000 spp.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "gpurun_out/ev_$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
run bench 400 python bench.py
run b1x100 400 python bench.py --nfb 1 --spp 100 --no-cpu-baseline
run b2host 400 python bench.py --gpus 2 --gather host --no-cpu-baseline
run c5full 600 python bench.py --scene final --width 3840 --height 2159 --nfb 100 --spp 100 --steps 1 --warmup 0 --cold-steps 1 --no-stats --no-cpu-baseline
grep -h '^{' gpurun_out/ev_*.log | cut -c1-400
