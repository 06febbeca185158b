"""Register / spill / scratch metadata of every render-kernel instantiation, from the AMDGPU
code-object metadata of a device-only assembly build of csrc/rt_kernels.hip.

usage: python scripts/isa_meta.py [OUT.txt] [-DNAME ...]
  (compiles with the product flags, ~60 s)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raytracing_gpu_amd import _build  # noqa: E402

FEAT = {0: "STATS", 1: "MOVING", 2: "RECT", 3: "TRI", 4: "LIST", 5: "XFORM", 6: "MEDIUM", 7: "CHECKER", 8: "NOISE",
        9: "IMAGE", 10: "BVH", 11: "EXACT", 12: "CHECK", 13: "LDS", 14: "STEP", 15: "WORLD", 16: "QLDS", 17: "MERGE", 18: "PROBE"}
NAMED = {25730: "C2 (SPHERES|LDS|STEP)", 1112: "C3 (CORNELL)", 1560: "C4 (MESH)", 1918: "C5 entry loop", 132990: "C5 (FINAL|MERGE)", 49268: "C3 world", 51070: "C5 world", 83480: "C4 quantized LDS",
         2046: "ALL"}


def main():
    argv = sys.argv[1:]
    extra = [a for a in argv if a.startswith("-D")]
    argv = [a for a in argv if not a.startswith("-D")]
    sys.argv = [sys.argv[0]] + argv
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "rt.s")
        flags = [f for f in _build.HIPCC_FLAGS if f not in ("-shared", "-fPIC")] + extra
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", "-o", s,
                        os.path.join(_build.CSRC, "rt_kernels.hip")], check=True, stderr=subprocess.DEVNULL)
        text = open(s).read()
    rows = []
    for blk in re.split(r"\n  - \.agpr_count:", text.split("amdhsa.kernels:", 1)[1]):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or "render" not in m.group(1):
            continue
        g = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))  # noqa: E731
        mask = int(re.search(r"ILi(\d+)E", m.group(1)).group(1))
        kind = "render_step_kernel" if "step" in m.group(1) else "render_kernel"
        feats = "|".join(v for b, v in FEAT.items() if mask >> b & 1)
        rows.append((kind, mask, g("vgpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"),
                     g("private_segment_fixed_size"), NAMED.get(mask & ~1, ""), feats))
    rows.sort(key=lambda r: (r[0], r[1]))
    out = [f"# build_id {_build.kernel_build_id()}",
           "kernel                      vgprs  vgpr_spills  sgpr_spills  scratch_B  config  features"]
    for k, mask, v, vs, ss, priv, cfg, feats in rows:
        out.append(f"{k + '<' + str(mask) + '>':28s}{v:5d}  {vs:11d}  {ss:11d}  {priv:9d}  {cfg:22s}  {feats}")
    txt = "\n".join(out) + "\n"
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
