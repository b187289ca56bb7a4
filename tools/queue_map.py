#!/usr/bin/env python3
"""Hardware queues of the c2 dispatches in a rocprofv3 --kernel-trace directory of tools/c4_gap_probe.py part 5: the
dispatches come in blocks (one per stream kind, separated by idle gaps > 20 ms); per block, the queues its streams'
dispatches ran on and how many dispatches overlapped in time.  usage: queue_map.py <dir>"""
import collections
import csv
import glob
import json
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rt_render_kernel" in r["Kernel_Name"] and r["Grid_Size_X"] == "15360"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
blocks, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 20_000_000:
        blocks.append(cur)
        cur = []
    cur.append(b)
blocks.append(cur)
for i, bk in enumerate(blocks):
    sq = collections.Counter((r["Stream_Id"], r["Queue_Id"]) for r in bk)
    over = sum(1 for a, b in zip(bk, bk[1:]) if int(b["Start_Timestamp"]) < int(a["End_Timestamp"]))
    span = (int(bk[-1]["End_Timestamp"]) - int(bk[0]["Start_Timestamp"])) / 1e3
    print(json.dumps({"block": i, "dispatches": len(bk), "stream_queue": {f"{s}->{q}": n for (s, q), n in sq.items()},
                      "overlapping_pairs": over, "us_per_dispatch": round(span / len(bk), 2)}))
