#!/usr/bin/env python3
"""Microbenchmark of the eval-mode fused convolution (artsbir_conv2d_fwd_act:
folded-BN bias, Bottleneck residual add, ReLU in the epilogue) on the embed
leg's shapes, per forced tile configuration (ARTSBIR_PGEMM_CFG), next to a
plain copy of the residual into the output (the elementwise floor of the same
bytes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

SHAPES = [  # N, H, W, C, Co, R, residual
    (1152, 56, 56, 64, 256, 1, 1),
    (1152, 28, 28, 128, 512, 1, 1),
    (1152, 14, 14, 256, 1024, 1, 1),
    (1152, 7, 7, 512, 2048, 1, 1),
    (1152, 56, 56, 256, 64, 1, 0),
    (1152, 56, 56, 64, 256, 1, 0),
    (1152, 28, 28, 512, 128, 1, 0),
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
    only = os.environ.get("ONLY")
    shapes = [SHAPES[int(i)] for i in only.split(",")] if only else SHAPES
    for (N, H, W, C, Co, R, res) in shapes:
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, R, R, C, device=dev) * 0.05).bfloat16()
        bias = torch.randn(Co, device=dev) * 0.1
        y = torch.empty(N, H, W, Co, device=dev, dtype=torch.bfloat16)
        r = torch.randn(N, H, W, Co, device=dev).bfloat16() if res else None
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, R, 1, R // 2)
        nbytes = (x.numel() + y.numel() * (2 if res else 1)) * 2
        fl = 2.0 * N * H * W * C * Co * R * R
        t_c = timeit(lambda: y.copy_(r if res else y))
        print(f"== {N}x{H}x{W}x{C} -> {Co} {R}x{R} res{res}: {nbytes / 1e9:.2f} GB, {fl / 1e9:.0f} GFLOP; "
              f"copy of the output-sized tensor {t_c:.0f} us ({y.numel() * 4 / t_c / 1e3:.0f} GB/s)", flush=True)
        for cfg in os.environ.get("CFGS", "-2,0,1,2,3,4,5,10,11,15,20,21").split(","):
            os.environ["ARTSBIR_PGEMM_CFG"] = cfg
            try:
                t = timeit(lambda: _hip.call("artsbir_conv2d_fwd_act", d, x.data_ptr(), w.data_ptr(), y.data_ptr(),
                                             bias.data_ptr(), r.data_ptr() if res else None, 1 if res else 0, 1, st))
                kname = _hip.lib().artsbir_last_kernel().decode()
            except _hip.HipError as e:
                print(f"  cfg {cfg}: n/a ({str(e)[:60]})")
                continue
            print(f"  cfg {cfg:>2} {kname:28s} {t:8.1f} us ({nbytes / t / 1e3:6.0f} GB/s, {fl / t / 1e6:6.1f} TF)",
                  flush=True)
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)


if __name__ == "__main__":
    main()
