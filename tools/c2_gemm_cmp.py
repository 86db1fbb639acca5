#!/usr/bin/env python3
"""The C2 step's 1x1 convolutions as plain GEMMs (M = 1152 images x H x W
pixels, K = C in, N = C out, NHWC bf16): the library's forward conv (with the
per-segment BN statistics epilogue of the training forward, and the plain eval
form with bias + ReLU) next to torch.matmul (hipBLASLt) and a pure
read-A/write-C copy for scale.  For measurement only: the product path never
calls torch.matmul."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

SHAPES = [(56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128), (28, 256, 512),
          (14, 256, 1024), (14, 1024, 256), (14, 512, 1024), (7, 512, 2048), (7, 2048, 512), (7, 1024, 2048)]


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
    N = 1152
    for (H, C, Co) in SHAPES:
        M = N * H * H
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Co, 1, 1, C, device=dev) * 0.05).bfloat16()
        y = torch.empty(N, H, H, Co, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(3 * 2 * 32 * Co, device=dev)
        bias = torch.zeros(Co, device=dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, H, C, Co, 1, 1, 1, 0)
        fl = 2.0 * M * C * Co
        nb = 2.0 * (M * C + M * Co + C * Co)
        t_seg = timeit(lambda: _hip.call("artsbir_conv2d_fwd_seg", d, x.data_ptr(), w.data_ptr(), y.data_ptr(), 3,
                                         stats.data_ptr(), st))
        k_seg = _hip.lib().artsbir_last_kernel().decode()
        forced = []
        for c in os.environ.get("CANDS", "").split(","):
            if not c:
                continue
            os.environ["ARTSBIR_PGEMM_CFG"] = c
            try:
                tc = timeit(lambda: _hip.call("artsbir_conv2d_fwd_seg", d, x.data_ptr(), w.data_ptr(), y.data_ptr(),
                                              3, stats.data_ptr(), st))
                forced.append(f"c{c} {tc:.1f}")
            except _hip.HipError:
                forced.append(f"c{c} n/a")
            os.environ.pop("ARTSBIR_PGEMM_CFG")
        t_act = timeit(lambda: _hip.call("artsbir_conv2d_fwd_act", d, x.data_ptr(), w.data_ptr(), y.data_ptr(),
                                         bias.data_ptr(), None, 0, 1, st))
        k_act = _hip.lib().artsbir_last_kernel().decode()
        a2, b2, c2 = x.view(M, C), w.view(Co, C), y.view(M, Co)
        t_lib = timeit(lambda: torch.matmul(a2, b2.t(), out=c2))
        src = torch.empty(M * Co, device=dev, dtype=torch.bfloat16)
        t_cp = timeit(lambda: y.view(-1).copy_(src))  # write C + read an equal amount
        print(f"{H:3d}^2 {C:4d}->{Co:4d}  M={M:8d}  {fl / 1e9:6.1f} GF {nb / 1e9:5.2f} GB | "
              f"fwd_seg {t_seg:7.1f} us {nb / t_seg / 1e3:5.2f} TB/s {fl / t_seg / 1e6:6.1f} TF ({k_seg}) | "
              f"fwd_act {t_act:7.1f} us ({k_act}) | hipBLASLt {t_lib:7.1f} us {nb / t_lib / 1e3:5.2f} TB/s "
              f"{fl / t_lib / 1e6:6.1f} TF | copy(C) {t_cp:6.1f} us | forced: {', '.join(forced)}", flush=True)
        del x, w, y, src


if __name__ == "__main__":
    main()
