#!/bin/bash
# Round-3 profiles, part 1: GPU parity suite, then rocprofv3 trace + PMC passes for C2 and C3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -1 gpurun_out/tests.log; case $rc in 0) ;; *) exit $rc;; esac
NAME=c2 ARGS="--steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
NAME=c3 ARGS="--scene cornell_smoke --width 800 --height 800 --steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
