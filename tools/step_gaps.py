#!/usr/bin/env python3
"""Where the C2 step's wall time goes beyond the main stream's kernels: one
profiled step with every library launch bracketed by HIP events (the bench's
_hip.PROFILE mode), placed on a common clock (elapsed time from a reference
event), then per stream the busy time, and on the main stream the idle gaps
(> --gap us) with the launch that ended each one — the final join with the
weight-gradient stream shows as the gap before the optimizer.

    python tools/step_gaps.py [--batch 384] [--gap 20] [--tune-cache F] [--mode overlap|skip|serial]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=384)
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--tune-cache", default=os.path.join(ROOT, "profiles", "tune_r5.txt"))
    ap.add_argument("--mode", default="overlap", choices=["overlap", "skip", "serial"])
    ap.add_argument("--side-tail", type=int, default=25, help="side-stream launches listed after main's last one")
    ap.add_argument("--by-tag", type=int, default=0, help="also list the N largest (kernel, tag) groups")
    ap.add_argument("--pre", type=int, default=0, help="steps enqueued (no sync) before the profiled one")
    ap.add_argument("--host", action="store_true", help="main-stream launches the GPU reached before the host issued them")
    args = ap.parse_args()
    import _hip
    import bench
    import engine
    engine.SKIP_WGRAD[0] = args.mode == "skip"
    engine.OVERLAP_WGRAD = args.mode != "serial"  # serial: the weight gradients in order on the main stream
    import losses
    import models
    import optim
    dev = torch.device("cuda:0")
    if args.tune_cache and os.path.exists(args.tune_cache):
        _hip.lib().artsbir_tune_load(args.tune_cache.encode())
    torch.manual_seed(1234)
    model = models.ModifiedResNet(bench.LAYERS, bench.OUT_DIM, heads=bench.HEADS, input_resolution=bench.RES,
                                  width=bench.WIDTH).to(dev)
    model.compute_dtype = torch.bfloat16
    model.train()
    opt = optim.Adam(model.parameters(), lr=1e-5, weight_decay=0.002)
    loss_fn = losses.TripletMarginLoss(margin=0.2)
    g = torch.Generator(device=dev).manual_seed(100)
    batch = [torch.randn(args.batch, 3, bench.RES, bench.RES, device=dev, generator=g) for _ in range(3)]
    main = torch.cuda.Stream(device=dev, priority=-1)
    torch.cuda.set_stream(main)

    def step():
        loss = loss_fn(*model.forward_branches(batch))
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    wall_plain = (time.perf_counter() - t0) * 1e3
    prof = []
    hts = [] if args.host else None
    _hip.HOST_TS = hts
    ref = torch.cuda.Event(enable_timing=True)
    ref.record()
    for _ in range(args.pre):  # the GPU is still busy with these when the profiled step is issued
        step()
    _hip.PROFILE = prof
    t0 = time.perf_counter()
    step()
    end = torch.cuda.Event(enable_timing=True)
    end.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    _hip.PROFILE = None
    _hip.HOST_TS = None
    main_id = main.cuda_stream
    rows = []
    for kname, fl, nb, e0, e1, tag, sid in prof:
        rows.append((ref.elapsed_time(e0), ref.elapsed_time(e1), kname, tag or "", sid))
    rows.sort()
    step_ms = ref.elapsed_time(end)
    print(f"step wall {wall_plain:.2f} ms (unprofiled), {wall:.2f} ms profiled; GPU span {step_ms:.2f} ms; mode {args.mode}")
    busy = collections.defaultdict(float)
    for s, e, k, t, sid in rows:
        busy[sid] += e - s
    for sid, b in busy.items():
        print(f"  stream {'main' if sid == main_id else hex(sid)}: kernels {b:.2f} ms")
    mrows = [r for r in rows if r[4] == main_id]
    gaps = []
    last = 0.0
    for s, e, k, t, sid in mrows:
        if s - last > args.gap / 1e3:
            gaps.append((s - last, last, k, t))
        last = max(last, e)
    tail = step_ms - last
    tot = sum(x[0] for x in gaps)
    print(f"  main idle gaps > {args.gap:.0f} us: {len(gaps)}, {tot:.2f} ms; after its last launch {tail:.2f} ms")
    for d, at, k, t in sorted(gaps, reverse=True)[:25]:
        print(f"    {d * 1e3:8.1f} us at {at:8.2f} ms before {k} [{t}]")
    srows = [r for r in rows if r[4] != main_id]
    if srows:
        lastmain_bwd = max(e for s, e, k, t, sid in mrows if not k.startswith("adam"))
        after = [r for r in srows if r[1] > lastmain_bwd]
        print(f"  side-stream work ending after the main stream's last kernel ({lastmain_bwd:.2f} ms): "
              f"{len(after)} launches, {sum(min(e - s, e - lastmain_bwd) for s, e, *_ in after):.2f} ms")
        for s, e, k, t, sid in after[:args.side_tail]:
            print(f"    {s:8.2f} - {e:8.2f} ms  {k:40s} {t}")
    if args.by_tag:
        _by_tag(rows, args.by_tag)
    if hts is not None and len(hts) == len(prof):
        # host issue time (ms from the step's start) vs the GPU start of the same
        # launch: where the GPU start is within 30 us after the host issue, the
        # stream was idle waiting for the host (host-bound stretch)
        t_host = [(h - t0) * 1e3 for h in hts]
        bound = []
        for (kname, fl, nb, e0, e1, tag, sid), th in zip(prof, t_host):
            if sid != main_id:
                continue
            tg = ref.elapsed_time(e0)
            if tg - th < 0.03:
                bound.append((th, tg, kname, tag or ""))
        print(f"  main-stream launches started within 30 us of their host issue: {len(bound)}")
        for th, tg, k, t in bound[:40]:
            print(f"    host {th:8.2f} ms  gpu {tg:8.2f} ms  {k:40s} {t}")


def _by_tag(rows, n):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for s, e, k, t, sid in rows:
        a = agg[(k, t)]
        a[0] += 1
        a[1] += e - s
    fam = collections.defaultdict(float)
    for (k, t), (c, ms) in agg.items():
        fam[t.split(" ")[0]] += ms
    print("  per tag family (ms): " + ", ".join(f"{f} {v:.2f}" for f, v in sorted(fam.items(), key=lambda x: -x[1])))
    for (k, t), (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:n]:
        print(f"    {ms:7.3f} ms {c:3d}x  {k:40s} {t}")


if __name__ == "__main__":
    main()
