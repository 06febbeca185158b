# round-4: GPU suite; same-box A/B of the deferred validation; strong-scaling estimates (C2, C5)
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
cat > /tmp/ab.txt <<'AB'
c5defer --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c5nodefer RT_HIP_LIB=build/ab/libnodefer.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c5defer_b --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c5nodefer_b RT_HIP_LIB=build/ab/libnodefer.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
timeout -k 10 300 python -u scripts/diag_scale.py > gpurun_out/scale_c2.log 2>&1; echo scale c2 rc=$?; cat gpurun_out/scale_c2.log
VERBOSE=1 timeout -k 10 400 python -u scripts/diag_scale.py final 3840 2159 100 1 > gpurun_out/scale_c5.log 2>&1; echo scale c5 rc=$?; grep "^N=" gpurun_out/scale_c5.log
export TMPDIR=/tmp; mkdir -p gpurun_out
b() { local name=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$name.log 2>&1; local rc=$?; echo "bench $name rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"cold_ms_per_step": [0-9.]*' gpurun_out/bench_$name.log | tr '\n' ' '; echo; case $rc in 0) ;; *) exit $rc;; esac; }
b bench
b 1x100 --nfb 1 --spp 100 --no-cpu-baseline
b c3 --scene cornell_smoke --width 800 --height 800 --no-cpu-baseline
b c4 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-cpu-baseline
b c5 --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-cpu-baseline
STEP_TIMEOUT=300 bash scripts/prof_all.sh || exit $?
