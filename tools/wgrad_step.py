#!/usr/bin/env python3
"""The C2 step's weight gradients one by one on an otherwise idle GPU: every conv
/ dense weight-gradient shape of ModifiedResNet((3,4,6,3), 512) at 3 x 384
images with its launches per step, timed with the committed tune table's choice
(ARTSBIR_TUNE_CACHE, default profiles/tune_r4.txt), and the per-step total: what
the side stream would cost if it ran alone.
    python tools/wgrad_step.py [tune_table]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

B = 1152
# (H, W input, C, Cout, R, stride, launches per step): stem, then layers 1-4
# (models.py:198-236, 300-330; Bottleneck conv1 / conv2 / conv3 / downsample)
CONV = [
    (224, 224, 8, 32, 3, 2, 1), (112, 112, 32, 32, 3, 1, 1), (112, 112, 32, 64, 3, 1, 1),
    (56, 56, 64, 64, 1, 1, 1), (56, 56, 256, 64, 1, 1, 2), (56, 56, 64, 64, 3, 1, 3), (56, 56, 64, 256, 1, 1, 4),
    (56, 56, 256, 128, 1, 1, 1), (56, 56, 128, 128, 3, 1, 1),
    (28, 28, 128, 512, 1, 1, 4), (28, 28, 256, 512, 1, 1, 1), (28, 28, 512, 128, 1, 1, 3), (28, 28, 128, 128, 3, 1, 3),
    (28, 28, 512, 256, 1, 1, 1), (28, 28, 256, 256, 3, 1, 1),
    (14, 14, 256, 1024, 1, 1, 6), (14, 14, 512, 1024, 1, 1, 1), (14, 14, 1024, 256, 1, 1, 5),
    (14, 14, 256, 256, 3, 1, 5), (14, 14, 1024, 512, 1, 1, 1), (14, 14, 512, 512, 3, 1, 1),
    (7, 7, 512, 2048, 1, 1, 3), (7, 7, 1024, 2048, 1, 1, 1), (7, 7, 2048, 512, 1, 1, 2), (7, 7, 512, 512, 3, 1, 2),
]
DENSE = [(57600, 4096, 2048, 1), (1152, 2048, 2048, 1), (1152, 512, 2048, 1)]  # attention pool: M, N(out), K(in)


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
    table = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("ARTSBIR_TUNE_CACHE",
                                                                   os.path.join(ROOT, "profiles", "tune_r4.txt"))
    _hip.lib().artsbir_tune_load(table.encode())
    dev = torch.device("cuda:0")
    st = _hip.stream()
    total, total_fl = 0.0, 0.0
    rows = []
    for (H, W, C, Co, R, s, n) in CONV:
        Ho, Wo = H // s, W // s
        x = torch.randn(B, H, W, C, device=dev).bfloat16()
        dy = torch.randn(B * Ho * Wo, Co, device=dev).bfloat16()
        dw = torch.zeros(Co, R * R * C, device=dev)
        d = _hip.conv_desc(torch.bfloat16, B, H, W, C, Co, R, R, s, R // 2)
        fl = 2.0 * B * Ho * Wo * C * Co * R * R
        us = timeit(lambda: _hip.call("artsbir_conv2d_wgrad", d, dy.data_ptr(), x.data_ptr(), None, None, 0,
                                      dw.data_ptr(), st))
        rows.append((f"conv {H}x{W} {C}->{Co} {R}x{R}/{s}", n, us, fl, _hip.lib().artsbir_last_kernel().decode()))
        del x, dy, dw
    for (M, N, K, n) in DENSE:
        dy = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        dw = torch.zeros(N, K, device=dev)
        us = timeit(lambda: _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dy.data_ptr(), N, x.data_ptr(), K,
                                      dw.data_ptr(), st))
        rows.append((f"dense M={M} {K}->{N}", n, us, 2.0 * M * N * K, _hip.lib().artsbir_last_kernel().decode()))
        del dy, x, dw
    for name, n, us, fl, kn in sorted(rows, key=lambda r: -r[1] * r[2]):
        total += n * us
        total_fl += n * fl
        print(f"{name:28s} x{n}  {us:8.1f} us  {n * us / 1e3:6.2f} ms/step  {fl / us / 1e6:6.1f} TF  {kn}", flush=True)
    print(f"total {total / 1e3:.2f} ms per step alone, {total_fl / total / 1e6:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
