#!/usr/bin/env python3
"""The pooled BatchNorm-backward passes alone (kind 1: the ReLU mask from the BN
parameters, pool 2: the gradient arrives at the 2x2-average-pooled resolution —
the bn2 backward of the strided Bottlenecks, models.py:205-213) at the C2 step's
shapes, three segments: artsbir_bn_bwd_reduce and artsbir_bn_bwd_apply, time and
HBM rate (reduce: d/4 + y, apply: d/4 + y + dy), to separate the kernels' own
rate from what they get inside the overlapped step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

# full-resolution y2 of the strided blocks' bn2 (layers 2, 3, 4) at 3 x 384 images
SHAPES = [(1152, 56, 56, 128), (1152, 28, 28, 256), (1152, 14, 14, 512)]


def best_of(fn, n=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    fn()
    torch.cuda.synchronize()
    for _ in range(n):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def main():
    dev = torch.device("cuda:0")
    st = _hip.stream()
    G = 3
    for (B, H, W, C) in SHAPES:
        Bs = B // G
        d = torch.randn(B, H // 2, W // 2, C, device=dev).bfloat16()
        y = torch.randn(B, H, W, C, device=dev).bfloat16()
        dy = torch.empty_like(y)
        prm = torch.randn(G, 4, C, device=dev)
        prm[:, 1] = prm[:, 1].abs() + 0.5
        coef = torch.randn(G, 3, C, device=dev)
        slots = torch.zeros(G, _hip.NSLOT, 2, C, device=dev)
        desc = _hip.BnBwdDesc()
        desc.dtype = _hip.DT_BF16
        desc.kind = 1
        desc.pool = 2
        desc.ntarget = 1
        desc.d = d.data_ptr()
        desc.mask_bn = prm.data_ptr()
        desc.y[0] = y.data_ptr()
        desc.mean[0] = prm[0, 0].data_ptr()
        desc.istd[0] = prm[0, 1].data_ptr()
        desc.slots[0] = slots.data_ptr()
        desc.coef[0] = coef.data_ptr()
        desc.dy[0] = dy.data_ptr()
        desc.B, desc.H, desc.W, desc.C = Bs, H, W, C
        desc.nseg = G
        desc.pstride = 4 * C
        desc.cstride = 3 * C
        desc.sstride = 2 * _hip.NSLOT * C
        tr = best_of(lambda: _hip.call("artsbir_bn_bwd_reduce", desc, st))
        ta = best_of(lambda: _hip.call("artsbir_bn_bwd_apply", desc, st))
        full = 2.0 * B * H * W * C
        nr, na = full / 4 + full, full / 4 + 2 * full
        print(f"pool2 k1 {B}x{H}x{W}x{C}: reduce {tr * 1e3:7.1f} us {nr / tr / 1e9:5.2f} TB/s | "
              f"apply {ta * 1e3:7.1f} us {na / ta / 1e9:5.2f} TB/s", flush=True)
        del d, y, dy


if __name__ == "__main__":
    main()
