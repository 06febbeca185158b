#!/bin/bash
# Round-3 profiles, part 2: rocprofv3 trace + PMC passes for C4 and C5.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NAME=c4 ARGS="--scene door --width 1920 --height 1079 --spp 16 --nfb 16 --steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
NAME=c5 ARGS="--scene final --width 3840 --height 2159 --spp 4 --nfb 4 --steps 2 --warmup 2 --cold-steps 1 --no-cpu-baseline" bash scripts/profile.sh || exit $?
