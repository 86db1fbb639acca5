#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes of bench.py.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python profiles/summarize_pmc.py gpurun_out profiles/r1_pmc_traffic.json

Counter values are KiB.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reports half the bytes of a wide coalesced stream -> doubled;
WRITE_SIZE is exact for 16-B-per-lane stores and float atomics.  Kernels are
keyed by the short names bench.py uses (template variants of one tile shape
are pooled, weighted by launch count).
"""
import collections
import csv
import json
import re
import sys


def short(name):
    m = re.match(r"_ZN7artsbir16conv_gemm_kernelIDF16bLi(\d+)ELi(\d+)E", name)
    if m:
        return f"conv_gemm_kernel<bf16,{m.group(1)},{m.group(2)}>"
    m = re.match(r"_ZN7artsbir16conv_gemm_kernelIfLi(\d+)ELi(\d+)E", name)
    if m:
        return f"conv_gemm_kernel<f32,{m.group(1)},{m.group(2)}>"
    m = re.match(r"_ZN7artsbir12wgrad_kernelIDF16bLi(\d+)ELi(\d+)E", name)
    if m:
        return f"wgrad_kernel<bf16,{m.group(1)},{m.group(2)}>"
    m = re.match(r"_ZN7artsbir12pgemm_kernelILi(\d+)ELi(\d+)E", name)
    if m:
        return f"pgemm_kernel<{m.group(1)},{m.group(2)}>"
    m = re.match(r"_ZN7artsbir14pstream_kernelILi(\d+)E", name)
    if m:
        return f"pstream_kernel<{m.group(1)}>"
    m = re.match(r"_ZN7artsbir13pwgrad_kernelILi(\d+)ELi(\d+)E", name)
    if m:
        return f"pwgrad_kernel<{m.group(1)},{m.group(2)}>"
    m = re.match(r"_ZN7artsbir\d+(\w+?_kernel)", name)
    if m:
        return m.group(1)
    return name.split("(")[0].replace("artsbir::", "")


def load(path, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += float(r["Counter_Value"]) * 1024.0
    return agg


def main(src, dst):
    fetch = load(f"{src}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = load(f"{src}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
    out = {}
    for k in fetch:
        if k not in write:
            continue
        nf, bf = fetch[k]
        nw, bw = write[k]
        out[k] = {"launches": nf, "fetch_bytes_per_launch": 2.0 * bf / nf, "write_bytes_per_launch": bw / nw,
                  "hbm_bytes_per_launch": 2.0 * bf / nf + bw / nw}
    out = dict(sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]))
    json.dump({"note": "FETCH_SIZE doubled (gfx950 correction), WRITE_SIZE as reported; bytes per launch",
               "kernels": out}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
