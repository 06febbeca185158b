# round-4 evidence: bench lines of C2-C5 (profiles/r04/bench_*.json via the merge), then rocprofv3
# kernel traces + PMC passes of the four workloads (scripts/prof_all.sh; scripts/prof_save.sh r04)
export TMPDIR=/tmp; mkdir -p gpurun_out
b() { local name=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$name.log 2>&1; local rc=$?; echo "bench $name rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"cold_ms_per_step": [0-9.]*' gpurun_out/bench_$name.log | tr '\n' ' '; echo; case $rc in 0) ;; *) exit $rc;; esac; }
b bench
b 1x100 --nfb 1 --spp 100 --no-cpu-baseline
b c3 --scene cornell_smoke --width 800 --height 800 --no-cpu-baseline
b c4 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-cpu-baseline
b c5 --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-cpu-baseline
STEP_TIMEOUT=300 bash scripts/prof_all.sh || exit $?
