#!/usr/bin/env python3
"""Per-kernel time in the last `frac` of a rocprofv3 kernel trace (the steady
passes of a repeated workload):  trace_window.py <kernel_trace.csv> <npasses>"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_steps import short  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
npass = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
cut = t1 - (t1 - t0) / npass  # the last pass (passes take about the same time once tuned)
agg = collections.defaultdict(lambda: [0.0, 0])
for r in rows:
    if int(r["Start_Timestamp"]) < cut:
        continue
    a = agg[short(r["Kernel_Name"])]
    a[0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    a[1] += 1
tot = sum(v[0] for v in agg.values())
print(f"window {(t1 - cut) / 1e6:.2f} ms, kernel time {tot:.2f} ms")
for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"  {ms:8.3f} ms {n:5d}x {1e3 * ms / n:9.1f} us  {k}")
