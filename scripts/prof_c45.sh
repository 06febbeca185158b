set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; echo "avail rc=$?"
NAME=c5 ARGS="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
NAME=c4 ARGS="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --steps 2 --warmup 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
