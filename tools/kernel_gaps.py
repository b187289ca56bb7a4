#!/usr/bin/env python3
"""Per-dispatch durations of rt_render_kernel and the idle gaps between consecutive dispatches, from a
rocprofv3 --kernel-trace directory.  usage: kernel_gaps.py <dir>"""
import csv
import glob
import json
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rt_render_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3 for i in range(len(rows) - 1)]
print(json.dumps({"dispatches": len(d), "kernel_us_median": round(statistics.median(d), 2),
                  "kernel_us_min": round(min(d), 2), "gap_us_median": round(statistics.median(gaps), 2),
                  "gap_us_max": round(max(gaps), 2)}))
