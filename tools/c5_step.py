#!/usr/bin/env python3
"""A few ViT-B/16 fp8 triplet steps at a given batch (profiling the C5 leg under rocprofv3)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import torch  # noqa: E402

import losses  # noqa: E402
import optim  # noqa: E402
import vit  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
mode = sys.argv[2] if len(sys.argv) > 2 else "fp8"
dev = torch.device("cuda", 0)
# ARTSBIR_TUNE_CACHE: autotuner choices loaded when the file exists, saved after
# the first step (a profiled re-run then launches no tuning trials)
tc = os.environ.get("ARTSBIR_TUNE_CACHE")
if tc and os.path.exists(tc):
    import _hip
    if _hip.lib().artsbir_tune_load(tc.encode()) < 0:
        raise RuntimeError(_hip.lib().artsbir_last_error().decode())
torch.manual_seed(1)
m = vit.VisionTransformer(224, 16, 768, 12, 12, 768).to(dev)
m.compute_dtype = {"fp8": "fp8", "bf16": torch.bfloat16}[mode]
opt = optim.Adam(m.parameters(), lr=1e-5)
loss_fn = losses.TripletMarginLoss(margin=0.2)
xs = [torch.randn(B, 3, 224, 224, device=dev) for _ in range(3)]
for it in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = m.forward_branches(xs)
    loss = loss_fn(*out)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    opt.zero_grad(set_to_none=False)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if it == 0 and tc:
        import _hip
        _hip.lib().artsbir_tune_save(tc.encode())
    print(f"step {it}: fwd {1e3 * (t1 - t0):.1f} ms, bwd+adam {1e3 * (t2 - t1):.1f} ms", flush=True)
