#!/usr/bin/env python3
"""Per-dispatch durations of rt_render_kernel, the gaps between consecutive dispatches and the per-frame
interval of the last `n` dispatches (the bench's timed steps), from a rocprofv3 --kernel-trace directory.
With frames in flight on several streams consecutive dispatches overlap (negative gaps): the interval,
(last end - first start) / n over the window, is then the per-frame throughput the bench's HIP events see.
usage: kernel_gaps.py <dir> [n]"""
import csv
import glob
import json
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rows = [r for r in csv.DictReader(open(f)) if "rt_render_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
d = [(e - s) / 1e3 for s, e in zip(st, en)]
gaps = [(st[i + 1] - en[i]) / 1e3 for i in range(len(rows) - 1)]
w = min(n, len(rows))
interval = (max(en[-w:]) - st[-w]) / 1e3 / w
print(json.dumps({"dispatches": len(d), "kernel_us_median": round(statistics.median(d), 2),
                  "kernel_us_min": round(min(d), 2), "kernel_us_median_last_n": round(statistics.median(d[-w:]), 2),
                  "gap_us_median": round(statistics.median(gaps), 2), "gap_us_max": round(max(gaps), 2),
                  "last_n": w, "interval_us_last_n": round(interval, 2)}))
