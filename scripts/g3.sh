# round-4: share tests, traversal diagnostics (world tree vs entry loop), C4/C5 profiles
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_shares_gpu.py -v --timeout 240 --timeout-method thread > gpurun_out/t_shares.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_shares.log | tail -30; echo shares rc=$rc; crash $rc && exit $rc
D="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --steps 1 --warmup 0 --cold-steps 1 --no-stats --no-cpu-baseline"
RT_HIP_LIB=build/ab/libdiag.so RT_WORLD_TREE=1 timeout -k 10 300 python bench.py $D > gpurun_out/diag_c5w.log 2>&1; echo diag c5w rc=$?
RT_HIP_LIB=build/ab/libdiag.so timeout -k 10 300 python bench.py $D > gpurun_out/diag_c5.log 2>&1; echo diag c5 rc=$?
RT_HIP_LIB=build/ab/libdiag.so timeout -k 10 300 python bench.py --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --steps 1 --warmup 0 --cold-steps 1 --no-stats --no-cpu-baseline > gpurun_out/diag_c4.log 2>&1; echo diag c4 rc=$?
grep -h "RT_STEP_DIAG\|value" gpurun_out/diag_c5w.log gpurun_out/diag_c5.log gpurun_out/diag_c4.log | cut -c1-220
STEP_TIMEOUT=300 NAME=c5 ARGS="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
STEP_TIMEOUT=300 NAME=c4 ARGS="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
