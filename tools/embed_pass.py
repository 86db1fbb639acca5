#!/usr/bin/env python3
"""A few eval-mode (inference) forward passes of the C2 encoder over 1152
images, for rocprofv3 kernel traces of the embed leg."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import models  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(1234)
m = models.ModifiedResNet(bench.LAYERS, bench.OUT_DIM, heads=bench.HEADS, input_resolution=bench.RES,
                          width=bench.WIDTH).to(dev)
m.compute_dtype = torch.bfloat16
m.eval()
x = [torch.randn(384, 3, 224, 224, device=dev) for _ in range(3)]
import _hip  # noqa: E402

with torch.no_grad():
    for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        m.forward_branches(x)
        torch.cuda.synchronize()
    if "--profile" in sys.argv:  # one more pass with per-launch HIP events, per (kernel, shape)
        prof = []
        _hip.PROFILE = prof
        m.forward_branches(x)
        torch.cuda.synchronize()
        _hip.PROFILE = None
        tot = 0.0
        rows = []
        for kname, fl, nb, e0, e1, tag in prof:
            ms = e0.elapsed_time(e1)
            tot += ms
            rows.append((ms, kname, tag, fl, nb))
        print(f"profiled launches {tot:.2f} ms")
        for ms, kname, tag, fl, nb in sorted(rows, reverse=True)[:40]:
            print(f"  {1e3 * ms:8.1f} us {nb / ms / 1e6 if ms else 0:7.0f} GB/s {fl / ms / 1e9 if ms else 0:7.1f} TF"
                  f"  {kname:32s} {tag}")
print("ok")
