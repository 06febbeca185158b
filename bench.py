#!/usr/bin/env python3
"""bench.py — Mrays/s (primary + bounces) of the gfx950 render path.

Default workload (BASELINE.json configs[1], C2): big_scene1 (the reference's random-spheres
scene, scenes.h:140-222), 1200x800, 100 rays per pixel split like the reference's main.cu as
no_fb = 10 frame buffers x 10 samples_per_pixel_per_fb (render.h:36-38), depth 50, seed 1984,
reference camera-RNG mode.  One step = one draw(): render_init + all 10 fb renders + per-fb
quantise/average (resolve) [+ the RCCL gather of the 8-bit rows to rank 0 when N > 1].
A ray segment = one top-level world query (render.h:63), counted on the device.

Every timed step is a ONE-SHOT draw (RT_FLAG_FRESH): the context forgets whatever it learned from
earlier draws of the same configuration, so each step runs as the reference's single draw() does --
the probe launch, the item schedule from its estimate, the render.  `value` and `ms_per_step` are
those draws.  The steady state of repeating one configuration (items claimed by the previous draw's
measured costs, split samples started from RNG states an earlier draw recorded) is reported beside
it as `warm_value` / `warm_ms_per_step`, never as `value`.

N > 1 (one process per GPU, torch.distributed over RCCL): rows are dealt in 4-row bands
round-robin over ranks; each rank renders and resolves its rows for every fb; one all-gather of
the 8-bit rows assembles the image.  Strong scaling (the image is fixed).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)
NODE_BYTES = 32         # rt_bvh_node
PRIM_BYTES = 48         # rt_prim
ITEM_BYTES = 32 + 12    # per (fb, pixel): RNG state read + fb write
F_LDS = 1 << 13          # variant feature bit: scene staged in LDS (rt_kernels.hip)
# LDS read roof: 256 B/clk/CU for ds_read_b64/b128 (MI355X_MICROARCH.md, LDS [CDNA4]) on
# 256 CUs at 2.4 GHz = 157.3 TB/s (the guide measures ~150 TB/s with every CU streaming).
LDS_PEAK_GBS = 256 * 256 * 2.4
# VALU issue roof: each of the 1024 SIMDs issues one wave64 VALU instruction every 2 cycles
# (32 lanes/clk: 157.3 TFLOP/s FP32 = 1024 x 32 x 2 x 2.4e9).
VALU_ISSUE_PER_S = 256 * 4 * 2.4e9 / 2


def lds_variant(kernel: str) -> bool:
    """The kernel name carries the variant's feature mask (rt_last_render_kernel): F_LDS set?"""
    try:
        return (int(kernel.rsplit("<", 1)[1].rstrip(">")) & F_LDS) != 0
    except (IndexError, ValueError):
        return False


def committed_pmc(workload: str, kernel: str):
    """PMC summary (scripts/profile.sh + scripts/pmc_summary.py) committed for this exact workload,
    kernel instantiation (variant mask included) and device-code build (kernel_build_id: hash of
    the flags and sources librt_hip.so is built from).  A summary of another build is never used:
    its counters would describe different code."""
    import glob

    from raytracing_gpu_amd._build import kernel_build_id

    bid = kernel_build_id()
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*_pmc.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("workload") == workload and d.get("kernel_full") == kernel and d.get("build_id") == bid
                and "hbm_bytes_per_launch" in d):
            best = (os.path.relpath(f, ROOT), d)
    return best, bid


def cpu_threads() -> tuple[int, int]:
    """(threads the CPU baseline uses, CPUs this process may run on).  The GPU box gives one GPU's
    job a 16-CPU share and exports OMP_NUM_THREADS=16 for it while sched_getaffinity still lists
    the whole machine; the baseline uses the share (the affinity count when no share is set)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(avail, share) if share > 0 else avail), avail


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default="big1")
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=10, help="samples_per_pixel_per_fb")
    ap.add_argument("--nfb", type=int, default=10, help="no_fb")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--cam", choices=["ref", "per_pixel"], default="ref")
    ap.add_argument("--band-rows", type=int, default=4, help="rows per band (800 rows = 200 bands: equal shares at N = 1, 2, 4, 8)")
    ap.add_argument("--exact", action="store_true", help="reference BVH visit set (no culling)")
    ap.add_argument("--no-lds", action="store_true", help="keep the scene in global memory")
    ap.add_argument("--no-step", action="store_true", help="segment-per-trip kernel even when the world is one BVH")
    ap.add_argument("--no-bins", action="store_true", help="camera rays traverse the BVH (no per-tile candidate lists)")
    ap.add_argument("--no-schedule", action="store_true", help="natural item order (no probe, no item schedule)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the untimed node/prim counting pass")
    ap.add_argument("--png", default="", help="write the assembled image (rank 0)")
    ap.add_argument("--warm-steps", type=int, default=5,
                    help="repeat draws timed after two priming draws (warm_*: the configuration's schedule and "
                         "split-sample states reused; 0 = skip)")
    ap.add_argument("--gather", default="rccl", choices=["rccl", "host"],
                    help="--gpus N without a launcher: ncclGather over distinct devices, or host copies (ranks may share a GPU)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="context option (include/rt_hip.h rt_ctx_options), e.g. --opt shade_min=52; "
                         "one-process-per-GPU path only")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="debug: gloo runs the N>1 path with host-side collectives and ranks sharing the visible GPUs")
    a = ap.parse_args()
    if a.steps < 1 or a.warmup < 0 or a.warm_steps < 0 or a.gpus < 1:
        ap.error("--steps and --gpus must be >= 1, --warmup and --warm-steps >= 0")
    return a


def parse_opts(items) -> dict:
    """--opt KEY=VALUE pairs -> rt_ctx_options fields (ints, or floats where the field is a float)."""
    out = {}
    for it in items:
        k, _, v = it.partition("=")
        out[k.strip()] = float(v) if any(ch in v for ch in ".e") else int(v)
    return out


CONFIG_OF = {"big1": "C2", "random": "C2", "cornell_smoke": "C3", "door": "C4", "final": "C5"}


def scene_assets(name: str):
    """Assets of the scenes that read files in the reference (kwargs for the product scene, kwargs
    for the oracle).  GPU boxes have no reference files: the door mesh comes from the committed
    assimp-import fixture (tests/golden/door_assimp.npz), textures are synthetic images of the real
    files' shapes (earthmap.jpg 3410x1518, Door_C.jpg 2048x2048)."""
    from raytracing_gpu_amd import assets

    if name == "earth":
        img = assets.synthetic_image(3410, 1518)
        return dict(images=[img]), dict(images=[img])
    if name in ("door", "cup", "final"):
        m = assets.door_mesh_from_fixture(os.path.join(ROOT, "tests", "golden", "door_assimp.npz"))
        imgs = [assets.synthetic_image(2048, 2048)] if name != "final" else [assets.synthetic_image(3410, 1518)]
        return dict(images=imgs, meshes=[m]), dict(images=imgs, meshes=[(m.tris, m.vertex_normals, m.image)])
    return {}, {}


def cpu_baseline(a, budget_s: float) -> dict:
    """The CPU oracle (C++ restatement of the reference render path) on the host's cores, over a
    bounded sample of the same workload: every k-th row, all fbs."""
    from oracle import ref_cpu

    threads, avail = cpu_threads()
    sc = ref_cpu.RefScene(a.scene, **scene_assets(a.scene)[1])
    cam = 0 if a.cam == "ref" else 1
    # calibrate on one row of fb 0
    t0 = time.perf_counter()
    _, c, _ = sc.render(a.width, a.height, a.spp, 0, a.depth, cam, rows=(a.height // 2, a.height), threads=threads)
    t1 = time.perf_counter() - t0
    per_row_fb = max(t1, 1e-4)  # one row runs on one thread; the sample spreads rows over `threads`
    nrows = max(1, min(a.height, int(budget_s * threads / (per_row_fb * a.nfb))))
    stride = max(1, a.height // nrows)
    segs = 0
    t0 = time.perf_counter()
    for f in range(a.nfb):
        _, c, _ = sc.render(a.width, a.height, a.spp, f, a.depth, cam, rows=(0, stride), threads=threads)
        segs += c["segments"]
    dt = time.perf_counter() - t0
    rows = len(range(0, a.height, stride))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": segs / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "host_cpus_visible": avail, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model,
            "sample": f"{a.scene} {a.width}x{a.height}, rows 0::{stride} ({rows} rows) x {a.nfb} fb x {a.spp} spp, "
                      f"{segs} segments in {dt:.1f} s, {threads} threads (oracle/ref_cpu.cpp, g++ -O2)"}


def roofline(a, stats, kname, avg_ms, rows, workload, world):
    """roofline object of the dominant kernel (render) from this run's live kernel time, the
    untimed stats pass's node/prim counts and, when committed for this exact build, its PMC summary."""
    if stats is None:
        return None
    items = a.nfb * rows * a.width
    bytes_launch = NODE_BYTES * stats["node_tests"] + PRIM_BYTES * stats["prim_tests"] + ITEM_BYTES * items
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
    # LDS / memory roof of the algorithmic bytes (node + primitive records + per-item
    # state and fb bytes).  The LDS variants read node/primitive records from the workgroup's
    # LDS copy of the scene, the others from L2 / HBM.
    mem = {"achieved": round(achieved, 2), "unit": "GB/s", "bytes_per_launch": int(bytes_launch),
           "bytes_per_segment": round(bytes_launch / max(stats["segments"], 1), 2),
           "node_tests_per_segment": round(stats["node_tests"] / max(stats["segments"], 1), 3),
           "prim_tests_per_segment": round(stats["prim_tests"] / max(stats["segments"], 1), 3),
           "counted_by": stats.get("kernel")}  # the F_STATS twin of the timed variant (same traversal)
    if lds_variant(kname):
        mem.update(served_from="LDS", peak=round(LDS_PEAK_GBS, 1), frac=round(achieved / LDS_PEAK_GBS, 4))
        roof = {"bound": "lds", "achieved": mem["achieved"], "peak": mem["peak"], "unit": "GB/s", "frac": mem["frac"]}
    else:
        # node/primitive records come from L2 (the scenes are a few MB): against the HBM peak the
        # ratio can exceed 1, so it is not reported as a roofline fraction; the binding roof needs
        # this build's PMC summary (below)
        mem.update(served_from="L2 (scene), HBM (RNG states, fb)", hbm_peak=HBM_PEAK_GBS,
                   ratio_to_hbm_peak=round(achieved / HBM_PEAK_GBS, 4))
        roof = {"bound": "unmeasured (no PMC summary for this build)", "achieved": None, "peak": None,
                "unit": None, "frac": None}
    roof.update({"traffic": None, "kernel": kname, "kernel_avg_ms": round(avg_ms, 3),
                 "fallbacks": stats["fallbacks"], "algorithmic": mem})
    pmc, bid = committed_pmc(workload, kname) if world == 1 else (None, None)
    roof["build_id"] = bid
    if pmc is not None:
        src, d = pmc
        # Counters are per launch of this same build and workload (rocprofv3 --pmc passes,
        # scripts/profile.sh); rates use this run's live kernel time.
        hbm = d["hbm_bytes_per_launch"]  # 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)
        roof["traffic"] = hbm
        roof["hbm"] = {"achieved": round(hbm / (avg_ms * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(hbm / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
        roof["pmc_source"] = src
        roof["pmc_git_head"] = d.get("git_head")
        roof["pmc_note"] = "counters committed for this build_id, measured in a separate rocprofv3 run, not this one"
        if "SQ_INSTS_VALU" in d:
            # binding roof of the megakernel: VALU issue (no MFMA: no dense contraction; the scene
            # is LDS/L2-resident, so HBM and the LDS array are far from their roofs)
            rate = d["SQ_INSTS_VALU"] / (avg_ms * 1e-3) / 1e9
            peak = VALU_ISSUE_PER_S / 1e9
            roof.update(bound="valu", achieved=round(rate, 2), peak=round(peak, 1),
                        unit="G wave64-VALU-inst/s", frac=round(rate / peak, 4))
            roof["valu"] = {"insts_per_launch": int(d["SQ_INSTS_VALU"]),
                            "lane_utilisation": round(d.get("valu_lane_utilisation", float("nan")), 4)}
            if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
                roof["valu"]["wait_any_share"] = round(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 4)
            if "SQ_LDS_BANK_CONFLICT" in d and "SQ_LDS_IDX_ACTIVE" in d:
                roof["valu"]["lds_bank_conflict_share"] = round(
                    d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1), 4)
    return roof


def workload_name(a) -> str:
    return (f"{CONFIG_OF.get(a.scene, 'scene')} {a.scene} {a.width}x{a.height}, {a.nfb} fb x {a.spp} spp = "
            f"{a.nfb * a.spp} rays/pixel, depth {a.depth}, cam {a.cam}, traversal {'exact' if a.exact else 'culled'}"
            f"{'' if not a.no_lds else ', global scene'}")


def out_line(a, value, world, dt_step, segs, roof, extra):
    out = {
        "metric": "Mrays/sec (primary+bounces) on RTIOW random-spheres 1200x800x100spp",
        "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt_step * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (reference scene generator, seed 1984)",
        "config": {"workload": workload_name(a),
                   "scene": a.scene, "width": a.width, "height": a.height, "rays_per_pixel": a.nfb * a.spp,
                   "no_fb": a.nfb, "spp_per_fb": a.spp, "max_depth": a.depth,
                   "segments_per_step": int(segs), "parallelism": f"rows{world}"},
        "roofline": roof,
    }
    out.update(extra)
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return main_inprocess(a)  # the C++ multi-GPU driver, one process, one thread per rank
    if a.gpus != world:
        raise SystemExit(f"bench.py --gpus {a.gpus} but WORLD_SIZE={world}")
    import torch
    import torch.distributed as dist

    import raytracing_gpu_amd as rt

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.backend == "gloo":  # rehearsal on fewer GPUs than ranks: ranks share devices
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(a.backend)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if a.backend == "gloo" else dev  # where collectives run

    ctx = rt.Context(local)
    opts = parse_opts(a.opt)
    if opts:
        ctx.set_options(**opts)
    sc = rt.Scene.builtin(a.scene, **scene_assets(a.scene)[0])
    ctx.upload(sc)
    cam = rt.RT_CAM_REF_SLOT0 if a.cam == "ref" else rt.RT_CAM_PER_PIXEL
    kw = dict(band_rows=a.band_rows, band_first=rank, band_stride=world, exact=a.exact, lds=not a.no_lds,
              step=not a.no_step, bins=not a.no_bins)
    args = rt.make_args(a.width, a.height, a.spp, 0, a.nfb, a.depth, cam, schedule=not a.no_schedule, **kw)
    cold_args = rt.make_args(a.width, a.height, a.spp, 0, a.nfb, a.depth, cam, schedule=not a.no_schedule,
                             fresh=True, **kw)
    rows = rt.owned_rows(args)
    all_rows = []
    for r in range(world):
        ar = rt.make_args(a.width, a.height, a.spp, 0, a.nfb, a.depth, cam, band_rows=a.band_rows,
                          band_first=r, band_stride=world)
        all_rows.append(rt.owned_rows(ar))
    max_rows = max(len(x) for x in all_rows)
    fb = torch.empty(a.nfb * len(rows) * a.width * 3, dtype=torch.float32, device=dev)
    img = torch.zeros(max_rows * a.width * 3, dtype=torch.uint8, device=dev)
    gathered = torch.empty(world * img.numel(), dtype=torch.uint8, device=cdev) if world > 1 else None

    seg_step = [0]
    kms, rms = [], []
    kname = [""]
    sched = []

    def step(args_):
        ctx.render_init(a.width, a.height, 1984)
        cnt = ctx.render(args_, fb.data_ptr())
        kms.append(ctx.last_kernel_ms())  # the render kernel alone (the roofline's launch duration)
        rms.append(ctx.last_render_ms())   # probe + schedule + render kernel
        kname[0] = ctx.last_render_kernel()
        sched.append(ctx.last_render_schedule())
        ctx.resolve(args_, fb.data_ptr(), img.data_ptr())
        if world > 1:
            dist.all_gather_into_tensor(gathered, img.to(cdev))
        seg_step[0] = cnt["segments"]
        return cnt

    def timed(n, args_):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            step(args_)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    # module load + first allocations, on a tiny image (a different configuration; the widest variant, so
    # that rocprof's statistics of the timed kernel hold the measured draws only)
    ctx.render_init(64, 36, 1984)
    tiny = rt.make_args(64, 36, 1, 0, 1, a.depth, cam, widest=True)
    tfb = torch.empty(64 * 36 * 3, dtype=torch.float32, device=dev)
    ctx.render(tiny, tfb.data_ptr())

    stats = None
    if not a.no_stats:  # untimed pass of the counting twin of the timed variant: node / prim tests for B_seg
        ctx.render_init(a.width, a.height, 1984)
        sargs = rt.make_args(a.width, a.height, a.spp, 0, a.nfb, a.depth, cam, band_rows=a.band_rows,
                             band_first=rank, band_stride=world, stats=True, exact=a.exact, lds=not a.no_lds,
                             step=not a.no_step, bins=not a.no_bins, schedule=False)
        stats = ctx.render(sargs, fb.data_ptr())
        stats["kernel"] = ctx.last_render_kernel()

    # warm leg (reported beside the value, never as it): two priming draws (the measuring one, the one
    # recording split-sample states), then repeats that reuse both
    dt_warm, warm_sched, warm_kms = None, [], None
    if a.warm_steps > 0:
        for _ in range(2):
            step(args)
        kms.clear()
        rms.clear()
        sched.clear()
        dt_warm = timed(a.warm_steps, args) / a.warm_steps
        warm_sched = sorted(set(sched))
        warm_kms = sum(kms) / len(kms)

    # the measured draws: one-shot (RT_FLAG_FRESH), W untimed then K timed -- last, so that a profile's
    # last K render dispatches are the timed ones (scripts/pmc_summary.py PMC_LAST)
    for _ in range(a.warmup):
        step(cold_args)
    kms.clear()
    rms.clear()
    sched.clear()
    dt = timed(a.steps, cold_args)
    assert all(x & (rt.RT_SCHED_PREVIOUS | rt.RT_SCHED_SPLIT_REPLAY) == 0 for x in sched), sched

    tot = torch.tensor([float(seg_step[0])], dtype=torch.float64, device=cdev)
    tmax = torch.tensor([dt, dt_warm or 0.0], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    segs = float(tot.item())
    dt, dt_warm = float(tmax[0].item()), (float(tmax[1].item()) if dt_warm is not None else None)
    value = segs * a.steps / dt / 1e6

    if rank == 0:
        avg_ms = sum(kms) / len(kms)
        workload = workload_name(a)
        roof = roofline(a, stats, kname[0], avg_ms, len(rows), workload, world)
        extra = {"kernel_ms": round(avg_ms, 3), "render_call_ms": round(sum(rms) / len(rms), 3),
                 "warm_value": round(segs / dt_warm / 1e6, 2) if dt_warm else None,
                 "warm_ms_per_step": round(dt_warm * 1e3, 3) if dt_warm else None,
                 "warm_kernel_ms": round(warm_kms, 3) if warm_kms else None,
                 "context_options": opts or "defaults",
                 "schedule": "value: one-shot draws (RT_FLAG_FRESH) -- nothing reused from an earlier draw, "
                             "each runs as a single draw() does: probe launch (bit 4), items ordered by its "
                             "estimate, render; warm_*: repeats of the configuration that reuse the previous "
                             "draw's measured item costs (bit 1) and recorded split-sample states (bit 2)",
                 "timed_schedule_bits": sorted(set(sched)), "warm_schedule_bits": warm_sched,
                 "stats_kernel": stats.get("kernel") if stats else None,
                 "driver": "torch.distributed (one process per GPU)" if world > 1 else "single process"}
        out = out_line(a, value, world, dt / a.steps, segs, roof, extra)
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a, a.cpu_seconds)
        print(json.dumps(out), flush=True)
        if a.png:
            from raytracing_gpu_amd import dist as rdist

            g = (gathered if world > 1 else img).cpu().numpy().reshape(world, max_rows, a.width, 3)
            rt.write_png(a.png, rdist.assemble(g, all_rows, a.height))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def main_inprocess(a):
    """`--gpus N` without a launcher: the product's C++ multi-GPU driver (librt_multi.so,
    include/rt_multi.h) in this one process -- one rt_ctx per device on its own host thread, row
    bands round-robin, ONE ncclGather of the 8-bit rows to rank 0 (RT_GATHER_RCCL, devices 0..N-1),
    host assembly.  `--gather host` lets N ranks share the visible GPUs (a rehearsal of the tiling
    on a one-GPU box; the rows are copied to the host instead of gathered over RCCL)."""
    import torch

    import raytracing_gpu_amd as rt
    from raytracing_gpu_amd import multi

    ndev = torch.cuda.device_count()
    if a.gather == "rccl":
        if ndev < a.gpus:
            raise SystemExit(f"--gpus {a.gpus}: {ndev} visible devices (RCCL needs one device per rank; "
                             "--gather host shares them)")
        devices = list(range(a.gpus))
        mode = multi.RT_GATHER_RCCL
    else:
        devices = [r % max(1, ndev) for r in range(a.gpus)]
        mode = multi.RT_GATHER_HOST
    m = multi.Multi(devices, mode)
    sc = rt.Scene.builtin(a.scene, **scene_assets(a.scene)[0])
    m.upload(sc)
    cam = rt.RT_CAM_REF_SLOT0 if a.cam == "ref" else rt.RT_CAM_PER_PIXEL
    kw = dict(band_rows=a.band_rows, exact=a.exact, lds=not a.no_lds, step=not a.no_step, bins=not a.no_bins)
    args = rt.make_args(a.width, a.height, a.spp, 0, a.nfb, a.depth, cam, schedule=not a.no_schedule, **kw)
    cold_args = rt.make_args(a.width, a.height, a.spp, 0, a.nfb, a.depth, cam, schedule=not a.no_schedule,
                             fresh=True, **kw)
    m.draw(rt.make_args(64, 36, 1, 0, 1, a.depth, cam, band_rows=4))  # module load on every device
    warms = []
    if a.warm_steps > 0:  # reported beside the value: repeats that reuse the schedule and split states
        for _ in range(2):
            m.draw(args)
        for _ in range(a.warm_steps):
            t0 = time.perf_counter()
            _, cnt, tm = m.draw(args)
            warms.append((time.perf_counter() - t0, tm))
    for _ in range(a.warmup):
        m.draw(cold_args)
    colds = []
    t0 = time.perf_counter()
    for _ in range(a.steps):  # one-shot draws; each is synchronous: every rank's stream and the gather drained
        img, cnt, tm = m.draw(cold_args)
        colds.append(tm)
    dt = time.perf_counter() - t0
    segs = cnt["segments"]
    value = segs * a.steps / dt / 1e6
    dt_warm = sum(x[0] for x in warms) / len(warms) if warms else None
    per_rank_k = [round(sum(t["kernel_ms"][r] for t in colds) / len(colds), 3) for r in range(a.gpus)]
    per_rank_warm = ([round(sum(t[1]["kernel_ms"][r] for t in warms) / len(warms), 3) for r in range(a.gpus)]
                     if warms else None)
    extra = {"warm_ms_per_step": round(dt_warm * 1e3, 3) if dt_warm else None,
             "warm_value": round(segs / dt_warm / 1e6, 2) if dt_warm else None,
             "kernel_ms_per_rank": per_rank_k, "warm_kernel_ms_per_rank": per_rank_warm,
             "render_ms_max": round(sum(t["render_ms_max"] for t in colds) / len(colds), 3),
             "gather_ms": round(sum(t["gather_ms"] for t in colds) / len(colds), 3),
             "gather_bytes": colds[-1]["gather_bytes"], "warm": colds[-1]["warm"],
             "schedule": "value: one-shot draws (RT_FLAG_FRESH), nothing reused from an earlier draw; warm_*: "
                         "repeats of the configuration that reuse the previous draw's item costs and "
                         "recorded split-sample states",
             "driver": f"librt_multi.so in one process, {a.gpus} ranks on devices {devices}, "
                       f"gather {'ncclGather (RCCL)' if mode == multi.RT_GATHER_RCCL else 'host copies'}; "
                       "a step includes the copy of the assembled image to the host"}
    out = out_line(a, value, a.gpus, dt / a.steps, segs, None, extra)
    print(json.dumps(out), flush=True)
    if a.png:
        rt.write_png(a.png, img)
    m.close()


if __name__ == "__main__":
    main()
