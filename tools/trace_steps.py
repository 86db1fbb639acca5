#!/usr/bin/env python3
"""Per-kernel time of the timed training steps from a rocprofv3 kernel trace of
bench.py: the steps are delimited by the adam_kernel dispatches (one per step);
the first `warmup` steps are skipped.

    python tools/trace_steps.py gpurun_out/prof/run_kernel_trace.csv [warmup] [--by-grid]
"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "")
    m = re.match(r"artsbir::(\w+)<([^()]*)>\(", n)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"_ZN7artsbir\d+(\w+?_kernel)I(.*?)EEv", n)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"_ZN7artsbir\d+(\w+?_kernel)", n)
    if m:
        return m.group(1)
    return n.split("(")[0].replace("artsbir::", "")[:60]


def main():
    path = sys.argv[1]
    warm = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 2
    by_grid = "--by-grid" in sys.argv
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    i0, i1 = adam[warm - 1] + 1, adam[-1] + 1
    steps = len(adam) - warm
    sel = rows[i0:i1]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        k = short(r["Kernel_Name"])
        if by_grid:
            k += f" grid={r['Grid_Size_X']}"
        a = agg[k]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy = sum(v[1] for v in agg.values())
    print(f"steps={steps} wall/step={(t1 - t0) / steps / 1e6:.2f} ms  kernel-busy/step={busy / steps / 1e6:.2f} ms")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{t / steps / 1e6:8.3f} ms  {n // steps:5d}/step  {t / n / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
