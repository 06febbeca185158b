#!/bin/bash
# rocprofv3 kernel trace + PMC passes (scripts/profile.sh) for the four bench workloads C2-C5.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NAME=c2 ARGS="--steps 2 --warmup 2 --warm-steps 2 --no-cpu-baseline" bash scripts/profile.sh || exit $?
NAME=c3 ARGS="--scene cornell_smoke --width 800 --height 800 --steps 2 --warmup 2 --warm-steps 2 --no-cpu-baseline" bash scripts/profile.sh || exit $?
NAME=c4 ARGS="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --steps 2 --warmup 2 --warm-steps 2 --no-cpu-baseline" bash scripts/profile.sh || exit $?
NAME=c5 ARGS="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --steps 2 --warmup 2 --warm-steps 2 --no-cpu-baseline" bash scripts/profile.sh || exit $?
