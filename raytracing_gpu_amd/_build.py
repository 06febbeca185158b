"""Build helpers: compile the gfx950 HIP library and the CPU oracle in-tree.

`build_hip()` produces raytracing_gpu_amd/librt_hip.so (hipcc --offload-arch=gfx950, host + device
code).  `build_oracle()` runs oracle/Makefile (test infrastructure only).
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "librt_hip.so")
MULTI_LIB = os.path.join(PKG, "librt_multi.so")
EXAMPLES = os.path.join(ROOT, "examples")
RT_MAIN = os.path.join(EXAMPLES, "bin", "rt_main")

HIP_SOURCES = ["rt_kernels.hip", "rt_scene.cpp", "rt_obj.cpp", "rt_image.cpp"]
# every header of csrc/ (rt_diag.h included): an edit to any of them rebuilds the library and changes
# kernel_build_id() (tests/test_build_cpu.py checks that each local #include is covered)
HIP_DEPS = HIP_SOURCES + sorted(f for f in os.listdir(CSRC) if f.endswith(".h"))
# -ffp-contract=off: no FMA contraction anywhere, so every float op rounds like the reference's
# C++ source and like the CPU oracle; fp32 div/sqrt correctly rounded (IEEE) on the device.
HIPCC_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math",
]


def kernel_build_id() -> str:
    """Identity of the device code: sha256 over the compile flags and every source the library is
    built from.  PMC summaries record it (scripts/pmc_summary.py) and bench.py uses a summary's
    counters only when the id matches the library it runs."""
    import hashlib

    h = hashlib.sha256(" ".join(HIPCC_FLAGS).encode())
    for f in HIP_DEPS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(ROOT, "include", "rt_hip.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_hip(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, f) for f in HIP_DEPS] + [os.path.join(ROOT, "include", "rt_hip.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *HIPCC_FLAGS, "-o", LIB + ".tmp", *[os.path.join(CSRC, f) for f in HIP_SOURCES]]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_multi(force: bool = False, verbose: bool = False) -> str:
    """librt_multi.so: the multi-GPU draw() (csrc/rt_multi.cpp, include/rt_multi.h), host C++ over
    librt_hip.so and RCCL (/opt/rocm/lib/librccl.so)."""
    deps = [os.path.join(CSRC, "rt_multi.cpp"), os.path.join(ROOT, "include", "rt_multi.h"), LIB]
    if not force and not _stale(MULTI_LIB, deps):
        return MULTI_LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "-o", MULTI_LIB + ".tmp", os.path.join(CSRC, "rt_multi.cpp"),
           "-L" + PKG, "-lrt_hip", "-lrccl", "-lpthread", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(MULTI_LIB + ".tmp", MULTI_LIB)
    return MULTI_LIB


def build_examples(force: bool = False, verbose: bool = False) -> str:
    """examples/bin/rt_main: the reference's main.cu as a C++ caller of include/rt_hip.h and
    include/rt_multi.h, linked against the in-tree libraries."""
    src = os.path.join(EXAMPLES, "rt_main.cpp")
    deps = [src, os.path.join(ROOT, "include", "rt_hip.h"), os.path.join(ROOT, "include", "rt_multi.h"), LIB, MULTI_LIB]
    if not force and not _stale(RT_MAIN, deps):
        return RT_MAIN
    os.makedirs(os.path.dirname(RT_MAIN), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-o", RT_MAIN + ".tmp", src,
           "-L" + PKG, "-lrt_hip", "-lrt_multi", "-Wl,-rpath,$ORIGIN/../../raytracing_gpu_amd", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=EXAMPLES)
    os.replace(RT_MAIN + ".tmp", RT_MAIN)
    return RT_MAIN


def build_oracle(force: bool = False) -> str:
    odir = os.path.join(ROOT, "oracle")
    args = ["make", "-C", odir, "-j4"]
    if force:
        subprocess.run(["make", "-C", odir, "clean"], check=True)
    subprocess.run(args, check=True, stdout=subprocess.DEVNULL)
    # the reference's own vendored stb_image, compiled where it lies (test pin for image decoding)
    if os.path.exists("/root/reference/external/stb_image.h"):
        subprocess.run(["make", "-C", odir, "ref"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(odir, "_build", "libref_cpu.so")


if __name__ == "__main__":
    build_hip(force="--force" in sys.argv, verbose=True)
    build_multi(force="--force" in sys.argv, verbose=True)
    build_examples(force="--force" in sys.argv, verbose=True)
    build_oracle(force="--force" in sys.argv)
    print(LIB)
