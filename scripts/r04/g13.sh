#!/bin/bash
# round-4: full GPU parity suite + smoke on the merged list-world search build, then C5's profile passes
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -1 gpurun_out/smoke.log; crash $rc && exit $rc
NAME=c5 ARGS="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" STEP_TIMEOUT=300 bash scripts/profile.sh
