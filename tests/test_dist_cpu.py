"""World-size-2 gloo test of the frame-buffer tiling + gather path (no GPU).

Each rank renders its 8-row bands of every fb with the CPU oracle standing in for the device
kernel (the oracle is the checker here, not the product), resolves them per pixel, all-gathers
the padded 8-bit rows and rank 0 assembles the image, which must equal a single-process draw().
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, NFB, BAND = 40, 29, 2, 3, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    from oracle import ref_cpu
    from raytracing_gpu_amd import dist as rdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = rdist.band_rows(H, BAND, rank, world)
    sc = ref_cpu.RefScene("big1")
    qs = []
    for f in range(NFB):
        fb = np.zeros(W * H * 3, np.float32)
        for j in rows:  # only this rank's rows
            sc.render(W, H, SPP, f, 50, 0, rows=(int(j), H), threads=1, fb=fb)
        qs.append(ref_cpu.quantize_fb(fb, W, H))
    img = ref_cpu.average(qs, W, H)            # PNG order; keep only our rows
    mine = img[H - 1 - rows]
    max_rows = max(len(r) for r in rdist.plan(H, BAND, world))
    t = torch.from_numpy(rdist.pad_rows(mine, max_rows).copy())
    out = torch.empty((world * max_rows,) + tuple(t.shape[1:]), dtype=torch.uint8)
    dist.all_gather_into_tensor(out, t)
    if rank == 0:
        q.put(rdist.assemble(out.numpy().reshape((world,) + tuple(t.shape)), rdist.plan(H, BAND, world), H))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_band_gather_matches_single_process(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue

    pic = None
    while pic is None:
        try:
            pic = q.get(timeout=5)
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), "a rank failed"
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want, _, _ = oracle.draw("big1", W, H, SPP, NFB)
    assert np.array_equal(pic, want)


def test_python_plan_matches_abi(rtlib):
    from raytracing_gpu_amd import dist as rdist

    for world in (1, 2, 3, 8):
        for r in range(world):
            a = rtlib.make_args(64, 1079, 1, band_rows=8, band_first=r, band_stride=world)
            assert np.array_equal(rtlib.owned_rows(a), rdist.band_rows(1079, 8, r, world))
