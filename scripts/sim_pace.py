"""Wave-level model of a stepwise launch (data: scripts/diag_order.py), for item orders.

scripts/sim_order.py models lanes at one pace.  Here a lane's pace per segment depends on how many
lanes of its own wave are busy (scripts/diag_pace.py on C2: 64 lanes 18.4 µs per
segment, 8 lanes 11.8, one lane 6.2 -- modelled as 6.2 + 2.05 log2(n) µs), every busy lane of a wave
advances one segment per wave step, and a wave refills its idle lanes from its claimed chunk of 64
positions (one chunk per work-counter claim, as claim_items).  The makespan is printed in ms for
orders built from the true costs or from the probe, and for the same orders with their first
waves * 64 positions "spread": position p takes rank (p % 64) * waves + p / 64, so each wave's first
chunk holds one item of every stratum of the ranking instead of 64 neighbouring ranks.

usage: sim_pace.py [--scale=X] build/orderdata/TAG [more tags]
"""
import heapq
import json
import math
import sys

import numpy as np

CUS, SIMDS, WAVES_PER_SIMD = 256, 4, 4


SCALE = 1.0  # --scale=X: paces of another scene (C4's full-wave pace is ~30 µs per segment: 1.63)


def pace_us(n):
    return SCALE * (6.2 + 2.05 * math.log2(n)) if n > 0 else 0.0


def makespan(cost_in_order, waves):
    """Event simulation: each wave steps its busy lanes one segment at pace_us(busy)."""
    c = np.asarray(cost_in_order, dtype=np.int64)
    n = len(c)
    nxt = 0  # global claim counter (positions)
    rem = [None] * waves
    chunk = [[0, 0] for _ in range(waves)]  # base, left
    heap = []

    def claim(w, k):
        nonlocal nxt
        got = []
        while k > 0:
            if chunk[w][1] == 0:
                if nxt >= n:
                    break
                chunk[w] = [nxt, 64]
                nxt += 64
            b, left = chunk[w]
            take = min(k, left)
            got.extend(range(b, min(b + take, n)))
            chunk[w] = [b + take, left - take]
            k -= take
        return got

    for w in range(waves):
        pos = claim(w, 64)
        rem[w] = c[pos].copy() if pos else np.zeros(0, dtype=np.int64)
        if len(rem[w]):
            heapq.heappush(heap, (0.0, w))
    end = 0.0
    while heap:
        t, w = heapq.heappop(heap)
        r = rem[w]
        busy = len(r)
        if busy == 0:
            end = max(end, t)
            continue
        # advance to the next item end in this wave at the current pace (batch of equal steps)
        k = int(r.min())
        t += k * pace_us(busy)
        r = r - k
        r = r[r > 0]
        idle = 64 - len(r)
        pos = claim(w, idle) if nxt < n or chunk[w][1] > 0 else []
        if pos:
            r = np.concatenate([r, c[pos]])
        rem[w] = r
        if len(r):
            heapq.heappush(heap, (t, w))
        end = max(end, t)
    return end / 1000.0


def spread(order, waves):
    k = min(len(order), waves * 64)
    p = np.arange(k)
    head = order[: (k // 64) * 64]
    nw = len(head) // 64
    p = np.arange(len(head))
    out = order.copy()
    out[: len(head)] = head[(p % 64) * nw + p // 64]
    return out


def stable_desc(keys):
    return np.argsort(-keys.astype(np.int64), kind="stable")


def main():
    global SCALE
    waves = CUS * SIMDS * WAVES_PER_SIMD
    for tag in sys.argv[1:]:
        if tag.startswith("--scale="):
            SCALE = float(tag.split("=", 1)[1])
            continue
        meta = json.load(open(tag + ".json"))
        d = np.load(tag + ".npz")
        W, spp, nfb = meta["W"], meta["spp"], meta["nfb"]
        rows = len(meta["rows"])
        items = rows * nfb * W
        cost = d["cost"].astype(np.int64)[:items]
        print(f"== {tag}: {items} items, {cost.sum()} segments, longest {cost.max()}; measured ms: "
              f"one-shot {[round(x[1], 2) for x in meta['product_cold']]}, natural "
              f"{[round(x[1], 2) for x in meta['natural']]}, warm {[round(x[1], 2) for x in meta['warm']]}", flush=True)
        q = np.arange(items) // (nfb * W)
        i = np.arange(items) % W
        raw = d["probe"][: rows * W].reshape(rows, W)
        g = np.minimum(raw, 10).astype(np.float64)
        r = 5
        pad = np.pad(g, r, mode="constant", constant_values=np.nan)
        h, w = g.shape
        sm = np.nanmean(np.stack([pad[dy:dy + h, dx:dx + w] for dy in range(2 * r + 1) for dx in range(2 * r + 1)]), 0)
        est = np.round(16 * sm)[q, i] * spp
        shift = 3
        while shift < 12 and ((32 * spp) >> shift) > 255:
            shift += 1
        orders = {
            "natural": np.arange(items),
            "true cost, 8-segment buckets": stable_desc(np.minimum(cost >> 3, 255)),
            "probe (r 5, depth 10)": stable_desc(np.minimum(est.astype(np.int64) >> (4 + shift), 255)),
        }
        for name, o in orders.items():
            print(f"  {name:34s} {makespan(cost[o], waves):7.3f} ms   spread {makespan(cost[spread(o, waves)], waves):7.3f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
