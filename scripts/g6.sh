# round-4: GPU suite, then A/B: deferred validation (C5), eager primitive loads (C2/C4), C3
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -20; echo all rc=$rc; crash $rc && exit $rc
cat > /tmp/ab.txt <<'AB'
c5defer --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c5nodefer RT_NO_DEFER=1 --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c2 --no-stats
c2eager RT_HIP_LIB=build/ab/libeager.so --no-stats
c4 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
c4eager RT_HIP_LIB=build/ab/libeager.so --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
c3 --scene cornell_smoke --width 800 --height 800 --no-stats
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
