#!/usr/bin/env python3
"""Microbenchmark of the weight-gradient kernels on the C2 step's shapes (conv
wgrads at 3 x 384 images) and the C5 projections (gemm_tn at 128 triplets),
per forced candidate (ARTSBIR_WGRAD_CFG) next to the tuned choice."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

B = 1152
CONV = [  # H, W (input), C, Cout, R, stride
    (56, 56, 64, 256, 1, 1),     # layer1 conv3 / downsample
    (56, 56, 256, 64, 1, 1),     # layer1 conv1
    (28, 28, 512, 128, 1, 1),    # layer2 conv1
    (14, 14, 256, 1024, 1, 1),   # layer3 conv3
    (7, 7, 2048, 512, 1, 1),     # layer4 conv1
    (56, 56, 64, 64, 3, 1),      # layer1 conv2
    (28, 28, 128, 128, 3, 1),    # layer2 conv2
    (14, 14, 256, 256, 3, 1),    # layer3 conv2
    (7, 7, 512, 512, 3, 1),      # layer4 conv2
    (56, 56, 128, 128, 3, 1),    # layer2 block-0 conv2 (before the 2x2 pool)
    (112, 112, 32, 32, 3, 1),    # stem conv2
    (112, 112, 32, 64, 3, 1),    # stem conv3
]
DENSE = [(75648, 2304, 768), (75648, 768, 768), (75648, 3072, 768), (75648, 768, 3072)]  # M, N(out), K(in)
# the folded BatchNorm backward's g^T x and x^T x per BN segment (artsbir_gemm_tn2,
# engine._wgrad_fold): M = 384 images' pixels, N1 = Co (g), N2 = K = Ci (x)
TN2 = [(301056, 512, 128), (301056, 512, 256), (75264, 1024, 256), (75264, 1024, 512), (18816, 2048, 512),
       (18816, 2048, 1024)]


def timeit(fn, reps=3):
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


def sweep(label, fl, run, ncand):
    os.environ.pop("ARTSBIR_WGRAD_CFG", None)
    t = timeit(run)
    kn = _hip.lib().artsbir_last_kernel().decode()
    res = [(t, "tuned:" + kn)]
    for c in list(range(ncand)) + [100, 101, 102]:  # then pw256 at its 3 split levels
        os.environ["ARTSBIR_WGRAD_CFG"] = str(c)
        try:
            t = timeit(run)
        except _hip.HipError:
            continue
        res.append((t, f"{c}:" + _hip.lib().artsbir_last_kernel().decode()))
    os.environ.pop("ARTSBIR_WGRAD_CFG", None)
    res.sort()
    print(f"== {label}: {fl / 1e9:.0f} GFLOP; tuned {res[[r[1].startswith('tuned') for r in res].index(True)][0]:.0f} us",
          flush=True)
    for t, name in res[:4]:
        print(f"   {t:8.1f} us {fl / t / 1e6:7.1f} TF  {name}", flush=True)


def main():
    dev = torch.device("cuda:0")
    st = _hip.stream()
    ncand = int(os.environ.get("NCAND", "40"))  # pwgrad tile configs x split levels + the four halo kernel variants (gemm.hip tune_wgrad)
    which = os.environ.get("WHICH", "conv,dense")
    if "conv" in which:
        only = os.environ.get("SHAPES")
        for ci, (H, W, C, Co, R, s) in enumerate(CONV):
            if only and str(ci) not in only.split(","):
                continue
            pad = R // 2
            Ho, Wo = H // s, W // s
            x = torch.randn(B, H, W, C, device=dev).bfloat16()
            dy = torch.randn(B * Ho * Wo, Co, device=dev).bfloat16()
            dw = torch.zeros(Co, R * R * C, device=dev)
            d = _hip.conv_desc(torch.bfloat16, B, H, W, C, Co, R, R, s, pad)
            fl = 2.0 * B * Ho * Wo * C * Co * R * R
            sweep(f"conv {B}x{H}x{W}x{C}->{Co} {R}x{R}/{s}", fl,
                  lambda: _hip.call("artsbir_conv2d_wgrad", d, dy.data_ptr(), x.data_ptr(), None, None, 0,
                                    dw.data_ptr(), st), ncand)
            del x, dy, dw
    if "tn2" in which:
        for (M, N1, K) in TN2:
            dy = torch.randn(M, N1, device=dev).bfloat16()
            x = torch.randn(M, K, device=dev).bfloat16()
            dw = torch.zeros(N1, K, device=dev)
            dw2 = torch.zeros(K, K, device=dev)
            fl = 2.0 * M * (N1 + K) * K
            sweep(f"tn2 M={M} {N1}+{K}x{K} ({M * (N1 + K) * 2 / 1e6:.0f} MB)", fl,
                  lambda: _hip.call("artsbir_gemm_tn2", _hip.DT_BF16, M, N1, K, K, dy.data_ptr(), N1, x.data_ptr(), K,
                                    x.data_ptr(), K, dw.data_ptr(), dw2.data_ptr(), st), ncand)
            del dy, x, dw, dw2
    if "dense" in which:
        for (M, N, K) in DENSE:
            dy = torch.randn(M, N, device=dev).bfloat16()
            x = torch.randn(M, K, device=dev).bfloat16()
            dw = torch.zeros(N, K, device=dev)
            fl = 2.0 * M * N * K
            sweep(f"dense M={M} {N}x{K}", fl,
                  lambda: _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dy.data_ptr(), N, x.data_ptr(), K,
                                    dw.data_ptr(), st), ncand)
            del dy, x, dw


if __name__ == "__main__":
    main()
