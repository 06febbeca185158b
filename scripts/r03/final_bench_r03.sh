export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/fb_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-cpu-baseline > gpurun_out/fb_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --nfb 1 --spp 100 --no-cpu-baseline > gpurun_out/fb_1x100.log 2>&1 && \
timeout -k 10 300 python -u bench.py --scene final --width 3840 --height 2159 --spp 100 --nfb 100 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/fb_c5full.log 2>&1
