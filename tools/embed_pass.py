#!/usr/bin/env python3
"""bench.py's embed leg alone (C2 ModifiedResNet, eval BatchNorm, 3 x 384 images
per pass) for rocprofv3 PMC passes: with ARTSBIR_TUNE_CACHE set, the autotuner's
choices are loaded when the file exists and saved after the first (tuning) pass,
so a second, profiled run launches no tuning trials."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    import _hip
    import models
    dev = torch.device("cuda", 0)
    tc = os.environ.get("ARTSBIR_TUNE_CACHE")
    if tc and os.path.exists(tc) and _hip.lib().artsbir_tune_load(tc.encode()) < 0:
        raise RuntimeError(_hip.lib().artsbir_last_error().decode())
    torch.manual_seed(1234)
    model = models.ModifiedResNet(bench.LAYERS, bench.OUT_DIM, heads=bench.HEADS, input_resolution=bench.RES,
                                  width=bench.WIDTH).to(dev)
    model.compute_dtype = torch.bfloat16
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 384
    g = torch.Generator(device=dev).manual_seed(100)
    batch = [torch.randn(B, 3, bench.RES, bench.RES, device=dev, generator=g) for _ in range(3)]
    model.eval()
    with torch.no_grad():
        model.forward_branches(batch)
        torch.cuda.synchronize()
    if tc:
        _hip.lib().artsbir_tune_save(tc.encode())
    r = bench.embed_leg(model, batch, "bf16", 1, 3)
    print(json.dumps({k: r[k] for k in ("value", "ms_per_pass")}), flush=True)
