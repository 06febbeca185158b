# round-4 iteration: world-tree parity (shares), A/B bench of the list-world / quantized-LDS kernels, full GPU suite
export TMPDIR=/tmp; mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_shares_gpu.py -v --timeout 240 --timeout-method thread > gpurun_out/t_shares.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t_shares.log | tail -30; echo shares rc=$rc; crash $rc && exit $rc
cat > /tmp/ab.txt <<'AB'
c5w4 --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c5w3 RT_HIP_LIB=build/ab/libwpe3.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c5old RT_NO_WORLD_TREE=1 --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c3w --scene cornell_smoke --width 800 --height 800
c3old RT_NO_WORLD_TREE=1 --scene cornell_smoke --width 800 --height 800
c4q --scene door --width 1920 --height 1079 --spp 16 --nfb 16
c4old RT_NO_QLDS=1 --scene door --width 1920 --height 1079 --spp 16 --nfb 16
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_shares_gpu.py > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t_all.log | tail -30; echo all rc=$rc
