#!/bin/bash
# round-4 closing evidence (after the merged search, the triangle dedupe, the unrolled traversal
# loop and the scalar list loads): GPU suite, smoke, bench lines of C2-C5 (+ C5 at its configured
# 10 000 spp, one draw), then rocprofv3 traces + PMC passes (scripts/prof_all.sh); on the CPU side
# bash scripts/prof_save.sh r04_final and copy gpurun_out/bench_*.log lines into profiles/r04_final/
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -1 gpurun_out/smoke.log; crash $rc && exit $rc
b() { local name=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$name.log 2>&1; local rc=$?; echo "bench $name rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"cold_ms_per_step": [0-9.]*' gpurun_out/bench_$name.log | tr '\n' ' '; echo; case $rc in 0) ;; *) exit $rc;; esac; }
b bench
b 1x100 --nfb 1 --spp 100 --no-cpu-baseline
b c3 --scene cornell_smoke --width 800 --height 800 --no-cpu-baseline
b c4 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-cpu-baseline
b c5 --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-cpu-baseline
b c5full --scene final --width 3840 --height 2159 --spp 100 --nfb 100 --steps 1 --warmup 0 --cold-steps 1 --no-cpu-baseline --no-stats
STEP_TIMEOUT=300 bash scripts/prof_all.sh || exit $?
