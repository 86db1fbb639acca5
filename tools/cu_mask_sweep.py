#!/usr/bin/env python3
"""A/B of the weight-gradient stream's CU budget (engine.SIDE_CUS) on the C2
training step, in one process: ms/step for each K (0 = unrestricted)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402


def main():
    import bench
    import engine
    import losses
    import models
    import optim
    import _hip
    if os.path.exists(bench.TUNE_CACHE):  # the committed autotuner table, as bench.py loads it
        _hip.lib().artsbir_tune_load(bench.TUNE_CACHE.encode())
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    model = models.ModifiedResNet(bench.LAYERS, bench.OUT_DIM, heads=bench.HEADS, input_resolution=bench.RES,
                                  width=bench.WIDTH).to(dev)
    model.compute_dtype = torch.bfloat16
    model.train()
    opt = optim.Adam(model.parameters(), lr=1e-5, weight_decay=0.002)
    loss_fn = losses.TripletMarginLoss(margin=0.2)
    B = int(os.environ.get("BATCH", "384"))
    g = torch.Generator(device=dev).manual_seed(100)
    batch = [torch.randn(B, 3, bench.RES, bench.RES, device=dev, generator=g) for _ in range(3)]
    main_default = torch.cuda.Stream(device=dev, priority=-1)
    torch.cuda.set_stream(main_default)

    def step():
        loss = loss_fn(*model.forward_branches(batch))
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()

    step()
    ks = sys.argv[1:] or ["0", "64", "96", "128", "160", "192", "0"]
    for k in ks:
        # "xK": the side stream on K CUs and the main stream on every other CU
        # "xKs": the main stream on every CU but those K, weight gradients skipped
        # "cK": as "xK" with the side stream on mask bits 0..K-1 instead of spread CUs
        contig = k.startswith("c")
        split = k.startswith("x") or contig
        skip = split and k.endswith("s")
        if split:
            k = k[1:].rstrip("s")
        engine.SIDE_CONTIGUOUS[0] = contig
        torch.cuda.set_stream(engine.cu_masked_stream(dev, int(k), invert=True, contiguous=contig) if split
                              else main_default)
        # "skip": no weight gradients (the main stream alone); "serial": on the main stream
        engine.SKIP_WGRAD[0] = skip or k == "skip"
        engine.OVERLAP_WGRAD = k != "serial"
        engine.SIDE_CUS[0] = int(k) if k.isdigit() else 0
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 5
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        print(f"side CUs {('c' if contig else 'x' if split else '') + k + ('s' if skip else ''):>6}: {(time.perf_counter() - t0) / n * 1e3:8.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
