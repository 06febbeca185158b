"""Audit: culled vs exact traversal per BVH query over a workload; dumps disagreements."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import raytracing_gpu_amd as rt

scene = sys.argv[1] if len(sys.argv) > 1 else "big1"
W, H, spp, nfb = [int(x) for x in (sys.argv[2:6] if len(sys.argv) > 5 else (1200, 800, 10, 10))]
ctx = rt.Context(0)
ctx.upload(rt.Scene.builtin(scene))
ctx.render_init(W, H, 1984)
fb = torch.zeros(nfb * H * W * 3, dtype=torch.float32, device="cuda")
c = ctx.render(rt.make_args(W, H, spp, 0, nfb, 50, 0, audit=True), fb.data_ptr())
n, log = ctx.audit_log()
print("segments", c["segments"], "disagreements", n)
np.set_printoptions(precision=9, suppress=False, linewidth=200)
for e in log[:40]:
    ii = e.view(np.int32)
    print("o", e[0:3], "d", e[3:6], "tm %.6f" % e[6], "tmin %g tmax %g" % (e[7], e[8]),
          "| culled t %.9g prim %d rank %d | exact t %.9g prim %d" % (e[9], ii[10], ii[13], e[11], ii[12]))
np.save("gpurun_out/audit_%s.npy" % scene, log)
