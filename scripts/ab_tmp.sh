set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; tail -1 gpurun_out/tests.log
timeout -k 10 300 python scripts/diag_launch.py 10 10
timeout -k 10 300 python scripts/diag_launch.py 100 1
RT_HIP_LIB=build/ab/libhost.so timeout -k 10 300 python scripts/diag_launch.py 10 10 | sed 's/^/host /'
