#!/usr/bin/env python3
"""Host enqueue time of the C2 training step vs its GPU time: is the Python /
ctypes launch path ever the bottleneck?  (bench.py's model, batch and step)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
import models  # noqa: E402
import optim  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(1234)
model = models.ModifiedResNet(bench.LAYERS, bench.OUT_DIM, heads=bench.HEADS, input_resolution=bench.RES,
                              width=bench.WIDTH).to(dev)
model.compute_dtype = torch.bfloat16
model.train()
opt = optim.Adam(model.parameters(), lr=1e-5, weight_decay=0.002)
loss_fn = losses.TripletMarginLoss(margin=0.2)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 384
batch = [torch.randn(B, 3, 224, 224, device=dev) for _ in range(3)]
torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))


def step():
    loss = loss_fn(*model.forward_branches(batch))
    opt.zero_grad(set_to_none=False)
    loss.backward()
    opt.step()
    return loss


for _ in range(3):
    step()
torch.cuda.synchronize()
for it in range(4):
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {it}: host enqueue {1e3 * (t1 - t0):.1f} ms, enqueue + drain {1e3 * (t2 - t0):.1f} ms", flush=True)
# back-to-back without a sync in between: the host runs ahead by at most the queue
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(4):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"4 steps back to back: host {1e3 * (t1 - t0) / 4:.1f} ms/step, total {1e3 * (t2 - t0) / 4:.1f} ms/step")
