"""CPU checks of the shared deterministic math (csrc/rt_detmath.h)."""
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_checker_sign_shortcut_matches_det_sinf(tmp_path):
    """sin_neg_fast == sign(det_sinf) on a strided sweep of every binade of 2^-20..2^17 (the
    exhaustive run, stride 1, checked all 620 756 994 floats: scripts/check_checker_sign.cpp)."""
    exe = tmp_path / "ccs"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    os.path.join(ROOT, "scripts", "check_checker_sign.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "97"], check=True, capture_output=True, text=True).stdout
    assert "mismatches 0" in out, out


def test_detmath_against_libm():
    """The deterministic definitions stay within a few float ulps of correctly rounded libm."""
    import ctypes

    src = os.path.join(ROOT, "raytracing_gpu_amd", "csrc", "rt_detmath.h")
    assert os.path.exists(src)
    from oracle import ref_cpu  # noqa: F401  (oracle builds with the same header)

    rng = np.random.default_rng(1)
    x = rng.uniform(-50, 50, 2000).astype(np.float32)
    # det_sinf is exercised through the oracle's checker texture; here check the header compiles
    # standalone and that sin values round like float(sin(double(x))) on a sample.
    code = r'''
#include "rt_detmath.h"
#include <cmath>
#include <cstdio>
int main(){ int bad=0; for(int i=-200000;i<=200000;++i){ float x=i*0.00037f;
  float a=rtm::det_sinf(x), b=(float)std::sin((double)x); float c=rtm::det_cosf(x), d=(float)std::cos((double)x);
  float l=rtm::det_logf(std::fabs(x)+1e-7f), m=(float)std::log((double)(std::fabs(x)+1e-7f));
  if (std::fabs(a-b)>2e-7f*std::fmax(1.f,std::fabs(b)) || std::fabs(c-d)>2e-7f*std::fmax(1.f,std::fabs(d)) ||
      std::fabs(l-m)>4e-7f*std::fmax(1.f,std::fabs(m))) ++bad; }
  printf("bad %d\n", bad); return bad!=0; }'''
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        cpp = os.path.join(d, "t.cpp")
        open(cpp, "w").write(code)
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.dirname(src), cpp,
                        "-o", os.path.join(d, "t")], check=True)
        out = subprocess.run([os.path.join(d, "t")], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout
