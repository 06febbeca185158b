#!/bin/bash
# One GPU-box session, the steps named in $STEPS (default: tests smoke bench), each under its own time
# limit; stops at the first crash-like exit (timeout, abort, segfault) and at a failed test run.
#   STEPS="tests c2 c4 scale_c4" bash scripts/gpu_round.sh
# Steps:
#   tests            pytest -m gpu (TESTS_K="expr" narrows it to pytest -k expr)
#   smoke            __graft_entry__.smoke()
#   c2 c2x100 c3 c3full c4 c5 c5full   bench.py lines of the BASELINE configs (C2 = the default)
#   scale_c2 scale_c2x100 scale_c4 scale_c5   scripts/diag_scale.py: every rank's share on this GPU
#                                      (SCALE_OPTS="--opt KEY=VALUE" passes context options)
#   trace_c2 trace_c4 trace_c5   scripts/trace_cold.sh: kernel timeline of one-shot draws (gaps = host waits)
#   osweep_c2 osweep_c2x100 osweep_c4 osweep_c5   scripts/diag_scale.py once per OSWEEP option setting
#   prof             scripts/prof_all.sh: rocprofv3 kernel traces + PMC passes of C2-C5
#   isa              scripts/isa_meta.py (registers / spills of every instantiation)
# BENCH_ARGS is appended to every bench line (e.g. BENCH_ARGS="--opt shade_min=52").
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
  tail -3 "gpurun_out/$name.log"
  if crash $rc; then echo "CRASH in $name, stopping"; exit $rc; fi
  return $rc
}
bench() {  # name args...
  local name=$1; shift
  run bench_$name 600 python -u bench.py "$@" ${BENCH_ARGS:-} || exit $?
  grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"warm_ms_per_step": [0-9.]*\|"warm_value": [0-9.]*\|"render_call_ms": [0-9.]*' \
    gpurun_out/bench_$name.log | tr '\n' ' '; echo
}
C4="--scene door --width 1920 --height 1079 --spp 16 --nfb 16"
C5="--scene final --width 3840 --height 2159 --spp 4 --nfb 4"
for s in ${STEPS:-tests smoke c2}; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    c2) bench c2 ;;
    c2x100) bench c2x100 --nfb 1 --spp 100 --no-cpu-baseline ;;
    c3) bench c3 --scene cornell_smoke --width 800 --height 800 --no-cpu-baseline ;;
    c3full) bench c3full --scene cornell_smoke --width 800 --height 800 --nfb 10 --spp 100 --steps 3 --warmup 2 --no-cpu-baseline ;;
    c4) bench c4 $C4 --no-cpu-baseline ;;
    c5) bench c5 $C5 --no-cpu-baseline ;;
    c5full) bench c5full --scene final --width 3840 --height 2159 --spp 100 --nfb 100 --steps 1 --warmup 0 --warm-steps 0 --no-cpu-baseline --no-stats ;;
    scale_c2) run scale_c2 600 python -u scripts/diag_scale.py big1 1200 800 10 10 ${SCALE_OPTS:-} || exit $? ;;
    scale_c4) run scale_c4 600 python -u scripts/diag_scale.py door 1920 1079 16 16 ${SCALE_OPTS:-} || exit $? ;;
    scale_c5) run scale_c5 600 python -u scripts/diag_scale.py final 3840 2159 4 4 ${SCALE_OPTS:-} || exit $? ;;
    scale_c2x100) run scale_c2x100 600 python -u scripts/diag_scale.py big1 1200 800 100 1 ${SCALE_OPTS:-} || exit $? ;;
    trace_c2) NAME=c2 bash scripts/trace_cold.sh || exit $? ;;
    btrace_c2) NAME=c2 bash scripts/trace_bench.sh || exit $? ;;
    trace_c4) NAME=c4 ARGS="--scene door --width 1920 --height 1079 --spp 16 --nfb 16" bash scripts/trace_cold.sh || exit $? ;;
    trace_c5) NAME=c5 ARGS="--scene final --width 3840 --height 2159 --spp 4 --nfb 4" bash scripts/trace_cold.sh || exit $? ;;
    osweep_*)  # scripts/diag_scale.py per context option setting: OSWEEP="probe_depth=0 probe_depth=8" STEPS=osweep_c2
      w=${s#osweep_}
      case $w in c2) wl="big1 1200 800 10 10";; c2x100) wl="big1 1200 800 100 1";; c4) wl="door 1920 1079 16 16";;
                 c3) wl="cornell_smoke 800 800 10 10";;
                 c5) wl="final 3840 2159 4 4";; *) echo "unknown workload $w"; exit 2;; esac
      for o in ${OSWEEP:-probe_depth=0}; do
        run osweep_${w}_${o//[=.,]/_} 600 python -u scripts/diag_scale.py $wl $(echo ",$o" | sed 's/,/ --opt /g') || exit $?
      done ;;
    prof) STEP_TIMEOUT=300 bash scripts/prof_all.sh || exit $? ;;
    isa) run isa 300 python scripts/isa_meta.py gpurun_out/isa_meta.txt || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
