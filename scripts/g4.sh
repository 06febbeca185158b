# round-4: parity suite, then A/B of the world tree (parked state) against the entry loop
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
cat > /tmp/ab.txt <<'AB'
c5w RT_WORLD_TREE=1 --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c5old --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c3w RT_WORLD_TREE=1 --scene cornell_smoke --width 800 --height 800
c3old --scene cornell_smoke --width 800 --height 800
c2 --no-stats
c4 --scene door --width 1920 --height 1079 --spp 16 --nfb 16
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
timeout -k 10 60 ./build/raycopy_copy > gpurun_out/raycopy.log 2>&1; echo raycopy_copy rc=$?
timeout -k 10 60 ./build/raycopy_inplace >> gpurun_out/raycopy.log 2>&1; echo raycopy_inplace rc=$?
cat gpurun_out/raycopy.log
