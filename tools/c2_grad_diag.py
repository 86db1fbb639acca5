#!/usr/bin/env python3
"""Diagnostic: where the f32 gradient of the C2 step (damped init, B=4) departs
from the float64 oracle — per parameter, and for the worst parameters per
output / input channel — next to the fp32 oracle's own error."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import test_c2_gpu as t  # noqa: E402
from oracle import encoder as oenc  # noqa: E402


def main():
    torch.set_num_threads(t._threads())
    dev = torch.device("cuda:0")
    el = oenc.synthetic_triplet(t.B, 224, seed=3)
    o64 = t._oracle_run(t.DAMP, el, torch.float64)
    o32 = t._oracle_run(t.DAMP, el, torch.float32)
    g64, g32 = o64["grad"], o32["grad"]
    import engine
    engine.set_deterministic(True)
    m = t._mine(dev, torch.float32)
    loss, embs, grads = t._step(m, el, dev)
    rows = []
    for k, gref in g64.items():
        sc = max(gref.abs().max().item(), 1e-30)
        rows.append(((grads[k] - gref).abs().max().item() / sc, (g32[k] - gref).abs().max().item() / sc, k))
    rows.sort(reverse=True)
    for e, e32, k in rows[:6]:
        d = (grads[k] - g64[k]).abs()
        d32 = (g32[k] - g64[k]).abs()
        print(f"{k}: mine {e:.3e} f32 {e32:.3e} shape {tuple(d.shape)}")
        if d.dim() >= 2:
            per_out = d.flatten(1).max(1).values
            per_in = d.flatten(2).max(2).values.max(0).values if d.dim() == 4 else d.max(0).values
            print("   worst out ch", per_out.topk(5).indices.tolist(), [f"{v:.2e}" for v in per_out.topk(5).values.tolist()],
                  "f32:", [f"{v:.2e}" for v in d32.flatten(1).max(1).values[per_out.topk(5).indices].tolist()])
            print("   worst in  ch", per_in.topk(5).indices.tolist(), [f"{v:.2e}" for v in per_in.topk(5).values.tolist()])
            print("   median out-ch err", f"{per_out.median().item():.2e}", "max|g|", f"{g64[k].abs().max().item():.2e}")
        else:
            print("   worst ch", d.topk(5).indices.tolist(), [f"{v:.2e}" for v in d.topk(5).values.tolist()],
                  "g64 there", [f"{v:.2e}" for v in g64[k][d.topk(5).indices].tolist()])


if __name__ == "__main__":
    main()
