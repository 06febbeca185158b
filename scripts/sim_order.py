"""Offline study of first-launch item orders (data: scripts/diag_order.py).

A launch is modelled as list scheduling: `lanes` lanes take items in claim order, each runs its item's
segments serially at one pace; the launch ends with its last lane.  For each order this prints the
makespan in units of the ideal (total segments / lanes) -- how far the longest chains that start late
stretch the launch.  Orders: natural (item index), the true costs (what a warm launch without split
samples uses), and probe estimates (grid step ps, smoothing radius, depth cap, cost buckets) as
rt_render builds them (probe_smooth_kernel, probe_keys_kernel).

usage: sim_order.py gpurun_out/order/TAG [more tags]
"""
import heapq
import json
import sys

import numpy as np

LANES = 256 * 1024


def makespan(cost_in_order, lanes=LANES):
    """Greedy list scheduling: each item goes to the lane that frees first."""
    c = np.asarray(cost_in_order, dtype=np.int64)
    n = len(c)
    if n <= lanes:
        return int(c.max())
    free = list(c[:lanes])
    heapq.heapify(free)
    for x in c[lanes:]:
        t = heapq.heappop(free)
        heapq.heappush(free, t + int(x))
    return max(free)


def stable_desc(keys):
    return np.argsort(-keys.astype(np.int64), kind="stable")


def smooth(grid, radius, agg="mean"):
    """Mean (or max) over a (2r+1)^2 window of the grid, clipped at the edges, in 1/16 units."""
    g = grid.astype(np.float64)
    if radius == 0:
        return np.round(16 * g)
    p = np.pad(g, radius, mode="constant", constant_values=np.nan)
    h, w = g.shape
    stack = [p[dy:dy + h, dx:dx + w] for dy in range(2 * radius + 1) for dx in range(2 * radius + 1)]
    s = np.stack(stack)
    return np.round(16 * (np.nanmax(s, axis=0) if agg == "max" else np.nanmean(s, axis=0)))


def main():
    for tag in sys.argv[1:]:
        meta = json.load(open(tag + ".json"))
        d = np.load(tag + ".npz")
        W, spp, nfb = meta["W"], meta["spp"], meta["nfb"]
        rows = len(meta["rows"])
        cost = d["cost"].astype(np.int64)
        items = rows * nfb * W
        cost = cost[:items]
        raw = d["probe"][: rows * W].reshape(rows, W)  # probe at every pixel (ps = 1), full depth
        ideal = cost.sum() / LANES
        q = np.arange(items) // (nfb * W)
        i = np.arange(items) % W
        print(f"== {tag}: {items} items, {cost.sum()} segments, ideal {ideal:.0f}, longest item {cost.max()}, "
              f"measured ms: product cold {meta['product_cold'][1]}, natural {meta['natural'][1]}, warm {meta['warm'][0][:2]}")

        def report(name, order):
            m = makespan(cost[order])
            print(f"  {name:42s} makespan {m:7d}  x{m / ideal:5.2f} ideal", flush=True)

        report("natural", np.arange(items))
        report("true cost, exact", stable_desc(cost))
        report("true cost, 8-segment buckets", stable_desc(np.minimum(cost >> 3, 255)))
        pix = cost.reshape(rows, nfb, W).mean(axis=1)  # the best any per-pixel estimate can know
        report("pixel mean of true costs (per-pixel ceiling)", stable_desc(np.round(pix[q, i] * 16).astype(np.int64)))
        for ps in (1, 2, 4):
            sub = raw[::ps, ::ps]
            for depth in (0, 10):
                g = np.minimum(sub, depth) if depth else sub
                for radius, agg in ((5, "mean"), (2, "mean"), (1, "max"), (0, "mean")):
                    v16 = smooth(g, radius, agg)
                    est = v16[q // ps, i // ps] * spp
                    shift = 3
                    while shift < 12 and ((32 * spp) >> shift) > 255:
                        shift += 1
                    key = np.minimum((est.astype(np.int64)) >> (4 + shift), 255)
                    report(f"probe ps={ps} depth={depth or 'full'} r={radius} {agg}", stable_desc(key))


if __name__ == "__main__":
    main()
