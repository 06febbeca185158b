export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shares_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_shares.log 2>&1; rc=$?; tail -3 gpurun_out/t_shares.log; echo shares rc=$rc
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_shares_gpu.py > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log; echo all rc=$rc
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-cpu-baseline --steps 3 > gpurun_out/b_c5.log 2>&1; echo c5 rc=$?; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/b_c5.log
