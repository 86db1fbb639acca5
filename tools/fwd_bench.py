#!/usr/bin/env python3
"""Microbenchmark of the forward convolution (BN statistics epilogue, three BN
segments) on the C2 step's HBM-bound shapes, per forced tile configuration
(ARTSBIR_PGEMM_CFG), next to a plain write / copy of the output for scale."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

SHAPES = [  # N, H, W, C, Co, R, stride
    (1152, 56, 56, 64, 256, 1, 1),
    (1152, 28, 28, 128, 512, 1, 1),
    (1152, 14, 14, 256, 1024, 1, 1),
    (1152, 7, 7, 512, 2048, 1, 1),
    (1152, 56, 56, 256, 64, 1, 1),
    (1152, 56, 56, 64, 64, 3, 1),
    (1152, 28, 28, 128, 128, 3, 1),
    (1152, 14, 14, 256, 256, 3, 1),
    (1152, 7, 7, 512, 512, 3, 1),
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
    only = os.environ.get("ONLY")  # comma-separated indices into SHAPES
    shapes = [SHAPES[int(i)] for i in only.split(",")] if only else SHAPES
    for (N, H, W, C, Co, R, s) in shapes:
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, R, R, C, device=dev) * 0.05).bfloat16()
        Ho, Wo = H // s, W // s
        y = torch.empty(N, Ho, Wo, Co, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(3, _hip.NSLOT, 2, Co, device=dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, R, s, R // 2)
        nbytes = (x.numel() + y.numel()) * 2
        fl = 2.0 * N * Ho * Wo * C * Co * R * R
        t_w = timeit(lambda: y.fill_(1.0))
        t_c = timeit(lambda: y.mul_(1.0))
        print(f"== {N}x{H}x{W}x{C} -> {Co} {R}x{R}/{s}: {nbytes / 1e9:.2f} GB, {fl / 1e9:.0f} GFLOP; "
              f"fill {t_w:.0f} us ({y.numel() * 2 / t_w / 1e3:.0f} GB/s), "
              f"rmw {t_c:.0f} us ({y.numel() * 4 / t_c / 1e3:.0f} GB/s)", flush=True)
        for cfg in os.environ.get("CFGS", "0,1,2,3,4,10,20,21").split(","):
            os.environ["ARTSBIR_PGEMM_CFG"] = cfg
            for with_stats in (1, 0):
                try:
                    t = timeit(lambda: _hip.call("artsbir_conv2d_fwd_seg", d, x.data_ptr(), w.data_ptr(),
                                                 y.data_ptr(), 3, stats.data_ptr() if with_stats else None, st))
                    kname = _hip.lib().artsbir_last_kernel().decode()
                except _hip.HipError as e:
                    print(f"  cfg {cfg}: n/a ({str(e)[:60]})")
                    break
                print(f"  cfg {cfg:>2} stats{with_stats} {kname:28s} {t:8.1f} us "
                      f"({nbytes / t / 1e3:6.0f} GB/s, {fl / t / 1e6:6.1f} TF)", flush=True)
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)


if __name__ == "__main__":
    main()
