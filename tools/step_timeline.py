#!/usr/bin/env python3
"""Timeline of the last full training step in a rocprofv3 kernel trace:
per-queue busy time, the union, and the step's tail (the kernels that run
after the main queue's last backward kernel, up to the optimizer).
    step_timeline.py <kernel_trace.csv> [step_marker_kernel=adam_kernel]"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_steps import short  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = short(r["Kernel_Name"])
rows.sort(key=lambda r: r["s"])
marks = [r for r in rows if marker in r["Kernel_Name"]]
if len(marks) < 2:
    sys.exit("fewer than two step markers")
t0, t1 = marks[-2]["e"], marks[-1]["e"]
step = [r for r in rows if r["s"] >= t0 and r["e"] <= t1]
qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
byq = collections.defaultdict(list)
for r in step:
    byq[r[qkey]].append(r)


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


print(f"step {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels")
print(f"  any queue busy {union([(r['s'], r['e']) for r in step]) / 1e6:.2f} ms")
for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    print(f"  queue {q}: {len(rs)} kernels, busy {union([(r['s'], r['e']) for r in rs]) / 1e6:.2f} ms, "
          f"first {(rs[0]['s'] - t0) / 1e6:.2f} last end {(max(r['e'] for r in rs) - t0) / 1e6:.2f} ms")
# phases: forward / backward split at the loss kernel, tail after the main queue's last non-optimizer kernel
mainq = max(byq, key=lambda q: len(byq[q]))
main = byq[mainq]
loss = [r for r in main if "triplet_fwd" in r["k"]]
if loss:
    print(f"  forward ends at {(loss[0]['e'] - t0) / 1e6:.2f} ms")
opt = [r for r in step if marker in r["Kernel_Name"]]
last_main = max((r["e"] for r in main if marker not in r["Kernel_Name"] and r["s"] < opt[-1]["s"]), default=t0)
print(f"  main queue's last kernel before the optimizer ends at {(last_main - t0) / 1e6:.2f} ms; "
      f"optimizer starts {(opt[-1]['s'] - t0) / 1e6:.2f} ms")
tail = [r for r in step if r["e"] > last_main and r["s"] < opt[-1]["s"]]
agg = collections.defaultdict(lambda: [0.0, 0])
for r in tail:
    a = agg[(r[qkey], r["k"])]
    a[0] += (min(r["e"], opt[-1]["s"]) - max(r["s"], last_main)) / 1e6
    a[1] += 1
print("  tail kernels (time inside the tail):")
for (q, k), (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:15]:
    print(f"    q{q} {ms:7.3f} ms {n:3d}x  {k}")
# the other queue over the backward: what overlaps what
for q, rs in byq.items():
    if q == mainq:
        continue
    ov = union([(max(r["s"], m["s"]), min(r["e"], m["e"])) for r in rs for m in main
                if min(r["e"], m["e"]) > max(r["s"], m["s"])])
    print(f"  queue {q} busy {union([(r['s'], r['e']) for r in rs]) / 1e6:.2f} ms, "
          f"of which overlapped with the main queue {ov / 1e6:.2f} ms")
