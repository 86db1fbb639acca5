#!/usr/bin/env python3
"""Per-launch profile of the C2 training step (bench.py's workload): every
library launch of the timed steps bracketed by HIP events, aggregated per
(kernel, shape tag) with algorithmic GB/s and TFLOP/s.

    python tools/step_profile.py [--batch 384] [--steps 2] [--tune-cache F]
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
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--tune-cache", default=None)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--mode", default="overlap", choices=["overlap", "serial", "skip"],
                    help="weight gradients overlapped (default), on the main stream, or left out (main stream alone)")
    args = ap.parse_args()
    import _hip
    import bench
    import engine
    engine.OVERLAP_WGRAD = args.mode == "overlap"
    engine.SKIP_WGRAD[0] = args.mode == "skip"
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
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(100)
    batch = [torch.randn(B, 3, bench.RES, bench.RES, device=dev, generator=g) for _ in range(3)]
    torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))

    def step():
        loss = loss_fn(*model.forward_branches(batch))
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()

    step()
    step()
    torch.cuda.synchronize()
    prof = []
    _hip.PROFILE = prof
    import time
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    _hip.PROFILE = None
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for kname, fl, nb, e0, e1, tag, *_ in prof:
        a = agg[(kname, tag)]
        a[0] += 1
        a[1] += e0.elapsed_time(e1) / 1e3
        a[2] += fl
        a[3] += nb
    tot = sum(v[1] for v in agg.values()) / args.steps
    print(f"step {el * 1e3:.2f} ms (wall), profiled launches {tot * 1e3:.2f} ms/step (event time, both streams)")
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for (k, tag), (n, s, fl, nb) in rows[:args.top]:
        print(f"{s / args.steps * 1e3:7.3f} ms  {n // args.steps:3d}x {s / n * 1e6:8.1f} us  "
              f"{nb / s / 1e9 if s else 0:7.1f} GB/s {fl / s / 1e12 if s else 0:7.1f} TF  {k:32s} {tag}")
    by_k = collections.defaultdict(float)
    for (k, _), v in agg.items():
        by_k[k] += v[1] / args.steps
    print("-- per kernel (ms/step):", ", ".join(f"{k} {v * 1e3:.2f}" for k, v in sorted(by_k.items(), key=lambda x: -x[1])))


if __name__ == "__main__":
    main()
