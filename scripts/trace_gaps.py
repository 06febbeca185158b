"""Timeline of the last one-shot draw in a rocprofv3 kernel trace: every kernel from the draw's
init_states_kernel on, its duration and the idle gap before it (host round trips show up as gaps).

usage: trace_gaps.py DIR   (rocprofv3 -d DIR -o run --output-format csv --kernel-trace)
"""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [k for k, r in enumerate(rows) if "init_states_kernel" in r["Kernel_Name"]]
for first, last in zip(starts[-3:], starts[-2:] + [len(rows)]):
    draw = rows[first:last]
    t0 = int(draw[0]["Start_Timestamp"])
    prev = t0
    print(f"--- draw from dispatch {draw[0]['Dispatch_Id']}")
    for r in draw:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:60]
        print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:9.1f} us  {name}")
        prev = e
    print(f"draw span {(prev - t0) / 1e3:.1f} us")
