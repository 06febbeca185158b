set -e
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "split" > gpurun_out/t_split.log 2>&1; tail -1 gpurun_out/t_split.log
for i in 1 2; do
  timeout -k 10 300 python scripts/diag_launch.py 100 1
  RT_HIP_LIB=build/ab/libhost.so timeout -k 10 300 python scripts/diag_launch.py 100 1 | sed 's/^/host /'
done
timeout -k 10 300 python scripts/diag_launch.py 10 10
