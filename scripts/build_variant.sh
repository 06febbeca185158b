#!/bin/bash
# Build an experiment variant of librt_hip.so with extra -D flags into build/ab/lib$NAME.so
#   bash scripts/build_variant.sh NAME [-DFOO ...]    (use with RT_HIP_LIB=build/ab/libNAME.so)
set -e
name=$1; shift
mkdir -p build/ab
cd raytracing_gpu_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math "$@" -o ../../build/ab/lib$name.so \
  rt_kernels.hip rt_scene.cpp rt_obj.cpp rt_image.cpp
