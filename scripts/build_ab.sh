#!/bin/bash
# Build an A/B library from another copy of rt_kernels.hip (the rest of csrc/ and include/ as in
# the tree) into build/ab/lib$NAME.so:   bash scripts/build_ab.sh NAME path/to/rt_kernels.hip [-DFOO ...]
set -e
name=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/raytracing_gpu_amd/csrc" "$tmp/include" "$root/build/ab"
cp "$root"/raytracing_gpu_amd/csrc/*.cpp "$root"/raytracing_gpu_amd/csrc/*.h "$tmp/raytracing_gpu_amd/csrc/"
cp "$root"/include/*.h "$tmp/include/"
cp "$src" "$tmp/raytracing_gpu_amd/csrc/rt_kernels.hip"
cd "$tmp/raytracing_gpu_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math "$@" -o "$root/build/ab/lib$name.so" \
  rt_kernels.hip rt_scene.cpp rt_obj.cpp rt_image.cpp
rm -rf "$tmp"
