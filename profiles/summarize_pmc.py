#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes of bench.py.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python profiles/summarize_pmc.py gpurun_out/pmc_train gpurun_out/pmc_retr profiles/r2_pmc_traffic.json

Counter values are KiB.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reports half the bytes of a wide coalesced stream -> doubled (exact
for 128-B requests only: a kernel whose loads make 64-B requests, such as
16 B x 4 lanes per row segment, is over-counted 2x by it; an optional third
pass pmc_req/ with TCC_EA0_RDREQ_32B/_64B/_128B and TCC_EA0_RDREQ gives the
read bytes by request size);
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
    bnb = ",bnb" if re.search(r"Lb1EEEv", name) else ""  # last template flag: fused BN backward
    # pgemm_kernel<BPX, BCH, WPX, WCH, NSTAGE, MULTI, BK, TWO, PF>: BK != 0 fused BN backward, PF prefetch
    m = re.match(r"_ZN7artsbir12pgemm_kernelILi(\d+)ELi(\d+)ELi\d+ELi\d+ELi\d+ELb[01]ELi(\d+)ELb[01]ELb([01])E", name)
    if m:
        return f"pgemm_kernel<{m.group(1)},{m.group(2)}{',bnb' if m.group(3) != '0' else ''}{',pf' if m.group(4) == '1' else ''}>"
    # pstream_kernel<BCH, WPX, WCH, NSTAGE, MULTI, BNB, FWDS>
    m = re.match(r"_ZN7artsbir14pstream_kernelILi(\d+)ELi\d+ELi\d+ELi\d+ELb[01]ELb([01])E", name)
    if m:
        return f"pstream_kernel<{m.group(1)}{',bnb' if m.group(2) == '1' else ''}>"
    m = re.match(r"_ZN7artsbir13pwgrad_kernelILi(\d+)ELi(\d+)E", name)
    if m:
        return f"pwgrad_kernel<{m.group(1)},{m.group(2)}>"
    m = re.match(r"_ZN7artsbir12sconv_kernelILi(\d+)ELi(\d+)ELi(\d+)E", name)
    if m:
        return f"sconv_kernel<{m.group(1)},{m.group(2)}{',s2' if m.group(3) == '2' else ''}{bnb}>"
    m = re.match(r"_ZN7artsbir12hconv_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])E", name)
    if m:
        return f"hconv_kernel<{m.group(1)},{m.group(2)},{m.group(3)}x{m.group(4)}{',bnb' if m.group(5) == '1' else ''}>"
    # BN-backward passes: <T, KIND, POOL, NT>, named by KIND as bench.py records
    # them (bn_bwd_apply_kernel<2>); rocprofv3 prints most of these launches with
    # a garbled demangling that keeps only the trailing arguments: ", EL, int, E,
    # NT>" is KIND 2 (after a fused dgrad), ", int, E, 2, 1>" KIND 1 with POOL 2
    m = re.match(r"_ZN7artsbir\d+(bn_bwd_(?:apply|reduce)_kernel)IDF16bLi(\d)E", name)  # mangled: KIND explicit
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    # (the apply forms only: counted against the launches bench.py records per
    # step — 46 of KIND 2, 4 of KIND 1 — the reduce forms are left generic)
    m = re.match(r"(?:void )?artsbir::bn_bwd_apply_kernel<bool _Accum, int, (EL, int, E, \d|E, 2, 1)>", name)
    if m:
        return f"bn_bwd_apply_kernel<{'2' if m.group(1).startswith('EL') else '1'}>"
    m = re.match(r"_ZN7artsbir\d+(\w+?_kernel)", name)
    if m:
        return m.group(1)
    # demangled form: void artsbir::name<a, b, ...>(args) -> exactly the names
    # bench.py records (the library's set_last_kernel strings)
    m = re.match(r"(?:void )?artsbir::(\w+_kernel)<([^>]*)>", name)
    if m:
        k, t = m.group(1), [x.strip() for x in m.group(2).split(",")]
        fb = ",bnb" if t[-1] == "true" and k == "sconv_kernel" else ""
        if k == "pgemm_kernel":  # <BPX, BCH, WPX, WCH, NSTAGE, MULTI, BK, TWO, PF, KS, GLB, X2>
            k32 = ",k32" if len(t) > 9 and t[9] == "32" else ""
            glb = ",glb" if len(t) > 10 and t[10] == "true" else ""
            fold = ",fold" if len(t) > 11 and t[11] == "true" else ""
            return f"{k}<{t[0]},{t[1]}{k32}{glb}{',bnb' if t[6] != '0' else ''}{',pf' if t[8] == 'true' else ''}{fold}>"
        if k == "pp256_kernel":  # <BK, TWO, TAPS, X2>
            tags = (["bnb"] if t[0] != "0" else []) + (["fold"] if len(t) > 3 and t[3] == "true" else [])
            return f"{k}<{','.join(tags)}>" if tags else k
        if k == "pwgrad_kernel":  # <BM, BN, WM, WN, NSTAGE, ...>: the 256 x 256 tiles carry their wave grid
            return f"{k}<{t[0]},{t[1]}{f',w{t[2]}x{t[3]}' if t[0] == t[1] == '256' else ''}>"
        if k == "hwgrad_kernel":  # <CT, OT, TR, NWC>: the 4-wave 64 x 64 variant is named w4
            return f"{k}<{t[0]},{t[1]}{',w4' if t[0] == t[1] == '64' and t[3] == '4' else ''}>"
        if k == "pw256_kernel":  # <DENSE>
            return f"{k}<{'dense' if t[0] == 'true' else 'conv'}>"
        if k == "pstream_kernel":  # <BCH, WPX, WCH, NSTAGE, MULTI, BNB, FWDS, BK, TWO, KS, X2, WGK>
            fold = ",fold" if len(t) > 10 and t[10] == "true" else ""
            fold += ",wg" if len(t) > 11 and t[11] not in ("0", "") else ""
            if len(t) > 9 and t[9] == "32":
                return f"{k}<{t[0]},k32>"
            if t[5] == "true":
                return f"{k}<{t[0]},{'bnbk' if len(t) > 7 and t[7] != '0' else 'bnb'}{fold}>"
            return f"{k}<{t[0]}{fold}>"
        if k == "hconv_kernel":
            return f"{k}<{t[0]},{t[1]},{t[2]}x{t[3]}{',bnb' if t[4] == 'true' else ''}>"
        if k == "sconv_kernel":
            return f"{k}<{t[0]},{t[1]}{',s2' if t[2] == '2' else ''}{fb}>"
        if k == "rstream_kernel":  # <K, BK, TWO>
            return f"{k}<bnb{',two' if len(t) > 2 and t[2] == 'true' else ''}>"
        return k
    return name.split("(")[0].replace("artsbir::", "").replace("void ", "")


def load(path, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += float(r["Counter_Value"]) * 1024.0
    return agg


def load_req(path):
    """read bytes by request size from a pass with TCC_EA0_RDREQ_{32B,64B,128B}
    and TCC_EA0_RDREQ: per kernel [dispatches, bytes = 32 n32 + 64 n64 + 128 n128,
    requests, RDREQ] (values summed over the counter's instances per dispatch)"""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        names[d] = short(r["Kernel_Name"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for d, c in per.items():
        a = agg[names[d]]
        a[0] += 1
        a[1] += 32 * c["TCC_EA0_RDREQ_32B"] + 64 * c["TCC_EA0_RDREQ_64B"] + 128 * c["TCC_EA0_RDREQ_128B"]
        a[2] += c["TCC_EA0_RDREQ_32B"] + c["TCC_EA0_RDREQ_64B"] + c["TCC_EA0_RDREQ_128B"]
        a[3] += c["TCC_EA0_RDREQ"]
    return agg


def summarize(src):
    fetch = load(f"{src}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = load(f"{src}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
    try:
        req = load_req(f"{src}/pmc_req/run_counter_collection.csv")
    except OSError:
        req = {}
    out = {}
    for k in fetch:
        if k not in write:
            continue
        nf, bf = fetch[k]
        nw, bw = write[k]
        out[k] = {"launches": nf, "fetch_bytes_per_launch": 2.0 * bf / nf, "write_bytes_per_launch": bw / nw,
                  "hbm_bytes_per_launch": 2.0 * bf / nf + bw / nw}
        if k in req and req[k][0]:
            n, b, nreq, rd = req[k]
            # FETCH_SIZE x 2 is exact only for 128-B requests; the request-size
            # counters give the read bytes whatever the access width
            out[k]["read_bytes_by_size_per_launch"] = b / n
            out[k]["hbm_bytes_by_size_per_launch"] = b / n + bw / nw
            out[k]["sized_requests_over_rdreq"] = round(nreq / rd, 4) if rd else None
    return out


def main(dst, *srcs):
    """srcs: run directories (each with pmc_fetch/ and pmc_write/); a kernel is
    taken from the first run that has it"""
    out = {}
    for src in srcs:
        for k, v in summarize(src).items():
            out.setdefault(k, v)
    out = dict(sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]))
    json.dump({"note": "FETCH_SIZE doubled (gfx950 correction), WRITE_SIZE as reported; with a third pass, "
                       "read bytes by request size (32/64/128-B TCC_EA0_RDREQ counters): hbm_bytes_by_size; "
                       "bytes per launch, "
                       "averaged over every launch of the kernel in the profiled runs (the training leg with "
                       "the autotune cache loaded: warmup + timed steps, no tuning trials)",
               "kernels": out}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[-1], *sys.argv[1:-1])
