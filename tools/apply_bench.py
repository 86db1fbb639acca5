#!/usr/bin/env python3
"""The BatchNorm-backward apply pass alone (artsbir_bn_bwd_apply, kind 2: g given,
one target, three segments) on the C2 step's activation shapes at 3 x 384 images:
time and HBM rate (read g and y, write dy: 6 bytes per element) per shape, to
separate the kernel's own rate from what it gets inside the overlapped step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

SHAPES = [(1152, 56, 56, 64), (1152, 56, 56, 256), (1152, 28, 28, 128), (1152, 28, 28, 512), (1152, 14, 14, 256),
          (1152, 14, 14, 1024), (1152, 7, 7, 512), (1152, 7, 7, 2048)]


def main():
    dev = torch.device("cuda:0")
    st = _hip.stream()
    G = 3
    for (B, H, W, C) in SHAPES:
        Bs = B // G
        g = torch.randn(B, H, W, C, device=dev).bfloat16()
        y = torch.randn(B, H, W, C, device=dev).bfloat16()
        dy = torch.empty_like(y)
        prm = torch.randn(G, 4, C, device=dev)
        prm[:, 1] = prm[:, 1].abs() + 0.5
        coef = torch.randn(G, 3, C, device=dev)
        desc = _hip.BnBwdDesc()
        desc.dtype = _hip.DT_BF16
        desc.kind = 2
        desc.pool = 0
        desc.ntarget = 1
        desc.d = g.data_ptr()
        desc.y[0] = y.data_ptr()
        desc.mean[0] = prm[0, 0].data_ptr()
        desc.istd[0] = prm[0, 1].data_ptr()
        desc.coef[0] = coef.data_ptr()
        desc.dy[0] = dy.data_ptr()
        desc.B, desc.H, desc.W, desc.C = Bs, H, W, C
        desc.nseg = G
        desc.pstride = 4 * C
        desc.cstride = 3 * C
        desc.sstride = 2 * _hip.NSLOT * C  # no slots in the apply; the check wants a whole block
        run = lambda: _hip.call("artsbir_bn_bwd_apply", desc, st)  # noqa: E731
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e30
        for _ in range(5):
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        nb = 6.0 * B * H * W * C
        print(f"apply k2 {B}x{H}x{W}x{C}: {best * 1e3:8.1f} us  {nb / best / 1e9:6.2f} TB/s  ({nb / 1e9:.2f} GB)",
              flush=True)
        del g, y, dy


if __name__ == "__main__":
    main()
