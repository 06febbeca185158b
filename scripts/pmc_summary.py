"""Summarise rocprofv3 PMC passes (scripts/profile.sh) for one kernel into a JSON file.

usage: pmc_summary.py OUT.json [kernel-substring] [workload] [name]

Reads gpurun_out/{name}_{fetch,write,sq,sq2,sq3,l2}/**/run_counter_collection.csv (name = "prof" by
default; scripts/profile.sh writes NAME_*), sums each counter per dispatch
of the kernel and averages over dispatches.  HBM traffic per launch follows the MI355X guide's
correction: FETCH_SIZE on gfx950 reports half the bytes of wide coalesced reads, so
traffic = 2 * FETCH_SIZE + WRITE_SIZE (both in KiB as rocprofv3 reports them).
Kernel durations come from gpurun_out/prof_trace/**/run_kernel_stats.csv.
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracing_gpu_amd._build import kernel_build_id  # noqa: E402

out = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "render_step_kernel<"
workload = sys.argv[3] if len(sys.argv) > 3 else ""
name = sys.argv[4] if len(sys.argv) > 4 else "prof"

res = {"kernel": kname, "workload": workload, "build_id": kernel_build_id(), "dispatches": {}}
try:
    res["git_head"] = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                     text=True).stdout.strip() or None
except OSError:
    res["git_head"] = None
# PMC_LAST=N: only the last N dispatches of the kernel in each pass (bench.py's timed steps; its
# earlier launches -- module load, cold draws, the measuring launch -- are other shapes or schedules)
last = int(os.environ.get("PMC_LAST", "0"))
res["dispatch_selection"] = f"last {last} dispatches of each pass (the timed steps)" if last else "all dispatches"
for p in (f"{name}_fetch", f"{name}_write", f"{name}_sq", f"{name}_sq2", f"{name}_sq3", f"{name}_l2"):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"gpurun_out/{p}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row.get("Kernel_Name", ""):
                continue
            per[row["Counter_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
    for c, d in per.items():
        keys = sorted(d)[-last:] if last else sorted(d)
        res[c] = sum(d[k] for k in keys) / len(keys)
        res["dispatches"][p] = len(keys)
for f in glob.glob(f"gpurun_out/{name}_trace/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if kname in row["Name"]:
            res.setdefault("trace", []).append({"name": row["Name"][:120], "calls": int(row["Calls"]),
                                                "avg_ms": float(row["AverageNs"]) / 1e6})
if last:  # the same dispatches' durations from the kernel trace
    for f in glob.glob(f"gpurun_out/{name}_trace/**/*kernel_trace.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if kname in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[-last:]]
        if durs:
            res["timed_dispatch_ms"] = [round(x, 4) for x in durs]
            res["timed_avg_ms"] = sum(durs) / len(durs)
names = {t["name"] for t in res.get("trace", [])}
if len(names) == 1:  # the full instantiation, e.g. render_step_kernel<25730>: bench.py matches on it
    n = names.pop()
    res["kernel_full"] = n.split("::", 1)[-1].split("(", 1)[0]
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    res["hbm_bytes_per_launch"] = int((2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024)
    res["hbm_correction"] = "2*FETCH_SIZE + WRITE_SIZE, KiB (MI355X_MICROARCH.md, HBM [CDNA4])"
if "SQ_THREAD_CYCLES_VALU" in res and "SQ_ACTIVE_INST_VALU" in res:
    # active lanes per VALU issue cycle / 64 (divergence measure)
    res["valu_lane_utilisation"] = res["SQ_THREAD_CYCLES_VALU"] / (64.0 * res["SQ_ACTIVE_INST_VALU"])
if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
    res["l2_hit_rate"] = res["TCC_HIT_sum"] / max(res["TCC_HIT_sum"] + res["TCC_MISS_sum"], 1.0)
if "SQ_WAIT_ANY" in res and "SQ_WAVE_CYCLES" in res:
    res["wait_any_share"] = res["SQ_WAIT_ANY"] / res["SQ_WAVE_CYCLES"]
if "SQ_LDS_BANK_CONFLICT" in res and "SQ_LDS_IDX_ACTIVE" in res:
    res["lds_bank_conflict_share"] = res["SQ_LDS_BANK_CONFLICT"] / max(res["SQ_LDS_IDX_ACTIVE"], 1.0)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "trace"}))
