#!/usr/bin/env python3
"""Microbenchmark of the conv GEMM variants on C2 shapes: forward, plain data
gradient and the fused BN-backward data gradient (kind 1 ACT, kind 3 RES with
residual), per forced tile configuration (ARTSBIR_PGEMM_CFG).  Env: CFGS (candidates),
SHAPES (indices into SHAPES)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

SHAPES = [  # N, H, W, C (dx channels), Co (dy channels), R, kind, res_mode
    (1152, 56, 56, 128, 128, 3, 1, 0),
    (1152, 28, 28, 128, 128, 3, 1, 0),
    (1152, 14, 14, 256, 256, 3, 1, 0),
    (1152, 14, 14, 1024, 256, 1, 3, 1),
    (1152, 28, 28, 512, 128, 1, 3, 1),
    (1152, 56, 56, 64, 256, 1, 1, 0),
    (1152, 56, 56, 256, 64, 1, 3, 1),
    (1152, 56, 56, 256, 128, 1, 3, 1),
]


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best * 1e3


def main():
    dev = torch.device("cuda:0")
    st = _hip.stream()
    only = os.environ.get("SHAPES")  # comma-separated indices into SHAPES (default: all)
    sel = [SHAPES[int(i)] for i in only.split(",")] if only else SHAPES
    for (N, H, W, C, Co, R, kind, rm) in sel:
        pad = R // 2
        G = 3
        x = torch.randn(N, H, W, Co, device=dev).bfloat16()      # dy (dgrad input, Co channels)
        w = (torch.randn(C, R, R, Co, device=dev) * 0.05).bfloat16()
        dx = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
        y = torch.randn(N, H, W, C, device=dev).bfloat16()
        res = torch.randn(N, H, W, C, device=dev).bfloat16() if rm else None
        bits = torch.randint(0, 255, (N * H * W * C // 8,), device=dev, dtype=torch.uint8)
        prm = torch.randn(G, 4, C, device=dev)
        prm[:, 1] = prm[:, 1].abs() + 0.5
        slots = torch.zeros(G, _hip.NSLOT, 2, C, device=dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, R, 1, pad)
        desc = _hip.BnBwdDesc()
        desc.dtype = _hip.DT_BF16
        desc.kind = kind
        desc.pool = 0
        desc.mask = bits.data_ptr() if kind == 3 else None
        desc.mask_bn = prm[0].data_ptr() if kind == 1 else None
        desc.ntarget = 1
        desc.y[0] = y.data_ptr()
        desc.mean[0] = prm[0, 0].data_ptr()
        desc.istd[0] = prm[0, 1].data_ptr()
        desc.slots[0] = slots.data_ptr()
        fl = 2.0 * N * H * W * C * Co * R * R
        nb = 2.0 * N * H * W * (Co + 2 * C + (C if rm else 0)) + (N * H * W * C / 8 if kind == 3 else 0)
        print(f"== dx {N}x{H}x{W}x{C} <- dy {Co} {R}x{R} kind{kind} res{rm}: {fl / 1e9:.0f} GFLOP", flush=True)
        for cfg in os.environ.get("CFGS", "0,1,2,3,10,21").split(","):
            os.environ["ARTSBIR_PGEMM_CFG"] = cfg
            try:
                t_plain = timeit(lambda: _hip.call("artsbir_conv2d_dgrad", d, x.data_ptr(), w.data_ptr(), dx.data_ptr(),
                                                   res.data_ptr() if rm else None, rm, st))
                t_bnb = timeit(lambda: _hip.call("artsbir_conv2d_dgrad_bnb", d, x.data_ptr(), w.data_ptr(),
                                                 dx.data_ptr(), res.data_ptr() if rm else None, rm, desc, G, 4 * C, st))
                kname = _hip.lib().artsbir_last_kernel().decode()
            except _hip.HipError as e:
                print(f"  cfg {cfg}: n/a ({str(e)[:60]})")
                continue
            print(f"  cfg {cfg:>2} {kname:28s} plain {t_plain:8.1f} us ({fl / t_plain / 1e6:6.1f} TF)  "
                  f"bnb {t_bnb:8.1f} us ({fl / t_bnb / 1e6:6.1f} TF, {nb / t_bnb / 1e3:6.0f} GB/s)", flush=True)
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)


if __name__ == "__main__":
    main()
