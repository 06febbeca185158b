#!/bin/bash
# Round-3 final build: C5 at its configured 10 000 spp (one cold draw, no stats pass), the in-process
# two-rank driver, then an A/B of the medium-record reload experiment.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "gpurun_out/fb_$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
run c5full 400 python -u bench.py --scene final --width 3840 --height 2159 --nfb 100 --spp 100 --steps 1 --warmup 0 --cold-steps 1 --no-stats --no-cpu-baseline
run b2host 300 python -u bench.py --gpus 2 --gather host --no-cpu-baseline
bash scripts/ab_env.sh < scripts/ab_park6.txt
