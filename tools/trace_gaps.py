#!/usr/bin/env python3
"""Timeline of one training step from a rocprofv3 --kernel-trace csv (every
kernel on the device, torch's own included): per queue the kernels in order,
their durations and the idle gaps between them, for the last complete step
(steps are delimited by the optimizer's pack_weights_kernel).

  python tools/trace_gaps.py <kernel_trace.csv> [--min-gap-us 10] [--window a:b]
"""
import argparse
import csv
import collections


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id") or r.get("Stream_Id") or "?"))
    rows.sort()
    return rows


def short(name):
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--min-gap-us", type=float, default=10.0)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    rows = load(args.csv)
    packs = [r for r in rows if "pack_weights_kernel" in r[2]]
    if len(packs) < 2:
        raise SystemExit("fewer than two pack_weights launches: no complete step")
    t0, t1 = packs[-2][1], packs[-1][1]  # from the end of one optimizer re-pack to the next
    step = [r for r in rows if t0 <= r[0] < t1 or r is packs[-1]]
    print(f"step: {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels")
    byq = collections.defaultdict(list)
    for r in step:
        byq[r[3]].append(r)
    qtime = {q: sum(e - s for s, e, _, _ in ks) for q, ks in byq.items()}
    main_q = max(qtime, key=lambda q: len(byq[q]))
    for q, ks in sorted(byq.items(), key=lambda kv: -qtime[kv[0]]):
        print(f"queue {q}: {len(ks)} kernels, {qtime[q] / 1e6:.3f} ms busy")
    # the device is idle when no queue runs a kernel
    busy = 0
    cur_s = cur_e = None
    idle = []
    for s, e, n, q in step:
        if cur_e is None:
            cur_s, cur_e = s, e
            continue
        if s > cur_e:
            busy += cur_e - cur_s
            idle.append((s - cur_e, cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"device busy {busy / 1e6:.3f} ms, idle {sum(i[0] for i in idle) / 1e6:.3f} ms in {len(idle)} gaps")
    print(f"largest device-idle gaps (before kernel):")
    for g, at, n in sorted(idle, reverse=True)[:args.top]:
        if g / 1e3 < args.min_gap_us:
            break
        print(f"  {g / 1e3:8.1f} us at {(at - t0) / 1e6:8.3f} ms  {short(n)}")
    # main-queue gaps (the queue with the most kernels) and what ran meanwhile elsewhere
    ks = byq[main_q]
    gaps = []
    for a, b in zip(ks, ks[1:]):
        if b[0] > a[1]:
            gaps.append((b[0] - a[1], a[1], a[2], b[2]))
    tot = sum(g[0] for g in gaps)
    print(f"main queue {main_q}: {len(gaps)} gaps, {tot / 1e6:.3f} ms idle")
    for g, at, pa, pb in sorted(gaps, reverse=True)[:args.top]:
        if g / 1e3 < args.min_gap_us:
            break
        print(f"  {g / 1e3:8.1f} us at {(at - t0) / 1e6:8.3f} ms  after {short(pa)[:45]:45s} before {short(pb)}")
    # kernels by name on the main queue
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n, q in ks:
        agg[short(n)][0] += 1
        agg[short(n)][1] += e - s
    print("main queue kernels by time:")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"  {t / 1e6:8.3f} ms {c:4d}x  {n}")


if __name__ == "__main__":
    main()
