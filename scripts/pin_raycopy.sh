#!/bin/bash
# Rebuild the round-2 "conditional ray copy" shape for ISA inspection (CPU only, no GPU):
# commit 9b8f2b5's kernel source with its in-place scatter reverted to the pre-fix form
# (`Ray sc; if (scatter(S, ray, h, a, sc, em, loc)) { ray = sc; ... }`, scatter force-inlined as
# in that commit), compiled for the widest variant render_kernel<2046> with the product flags,
# next to the fixed source.  Outputs: $OUT/{bug,fixed}.s and a -g build bugg.s whose .loc lines
# map the selects back to bug_rt_kernels.hip ("The conditional ray copy").
set -eu
OUT=${OUT:-/tmp/pin}
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT/a/b" "$OUT/include"
for f in rt_kernels.hip rt_detmath.h rt_xorwow.h rt_host_geom.h; do
  git -C "$REPO" show 9b8f2b5:raytracing_gpu_amd/csrc/$f > "$OUT/a/b/$f"
done
git -C "$REPO" show 9b8f2b5^:raytracing_gpu_amd/csrc/rt_kernels.hip > "$OUT/a/b/pre_rt_kernels.hip"
git -C "$REPO" show 9b8f2b5:include/rt_hip.h > "$OUT/include/rt_hip.h"
python3 - "$OUT/a/b" <<'EOF'
import sys
d = sys.argv[1]
s = open(f"{d}/rt_kernels.hip").read()
pre = open(f"{d}/pre_rt_kernels.hip").read()
a = s.index("template <int F>\n__device__ __forceinline__ bool scatter(const DScene& S, Ray& ray, const Hit& h, V& att, V& em, Rng& rng) {")
b = s.index("// ------------------------------------------------------------------ kernels", a)
pa = pre.index("template <int F>\n__device__ bool scatter(const DScene& S, const Ray& in, const Hit& h, V& att, Ray& out, V& em, Rng& rng) {")
pb = pre.index("// ------------------------------------------------------------------ kernels", pa)
s = s[:a] + pre[pa:pb].replace("__device__ bool scatter(", "__device__ __forceinline__ bool scatter(") + s[b:]
s = s.replace("if (scatter<F>(S, ray, h, a, em, loc)) {", "Ray sc;\n        if (scatter<F>(S, ray, h, a, sc, em, loc)) {\n          ray = sc;")
open(f"{d}/bug_rt_kernels.hip", "w").write(s)
EOF
cd "$OUT/a/b"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -DRT_ONLY_MASK=2046 --cuda-device-only -S"
/opt/rocm/bin/hipcc $FLAGS -o "$OUT/bug.s" bug_rt_kernels.hip 2>/dev/null
/opt/rocm/bin/hipcc $FLAGS -o "$OUT/fixed.s" rt_kernels.hip 2>/dev/null
/opt/rocm/bin/hipcc $FLAGS -g -o "$OUT/bugg.s" bug_rt_kernels.hip 2>/dev/null
echo "wrote $OUT/bug.s $OUT/fixed.s $OUT/bugg.s"
