#!/usr/bin/env python3
"""Weight-gradient candidate A/B (ARTSBIR_WGRAD_CFG forced) on the C2 / C5 wgrad
shapes, interleaved rounds in one process; torch fp32 on the same bf16 operands
checks the result (relative max error)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import torch  # noqa: E402

import _hip  # noqa: E402

CONV = [  # N, H, W, C, Cout, R (stride 1, pad R//2): C2's 3x3 convs and big 1x1 at 1152 images
    (1152, 56, 56, 64, 64, 3), (1152, 28, 28, 128, 128, 3), (1152, 14, 14, 256, 256, 3), (1152, 7, 7, 512, 512, 3),
    (1152, 56, 56, 128, 128, 3), (1152, 28, 28, 256, 256, 3), (1152, 14, 14, 1024, 256, 1), (1152, 56, 56, 64, 256, 1),
    (1152, 56, 56, 256, 64, 1), (1152, 56, 56, 256, 128, 1), (1152, 28, 28, 512, 128, 1), (1152, 28, 28, 128, 512, 1),
]
TN = [(302592, 768, 2304), (302592, 768, 768), (302592, 3072, 768), (302592, 768, 3072), (57600, 4096, 2048)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", default="auto,100,101,102")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    st = _hip.stream()
    jobs = []
    for N, H, W, C, Co, R in CONV:
        x = (torch.rand(N, H, W, C, device=dev) * 2 - 1).bfloat16()
        dy = (torch.rand(N, H, W, Co, device=dev) * 2 - 1).bfloat16()
        dw = torch.zeros(Co, R, R, C, device=dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, R, 1, R // 2)
        fl = 2.0 * N * H * W * Co * C * R * R

        def run(x=x, dy=dy, dw=dw, d=d):
            _hip.call("artsbir_conv2d_wgrad", d, dy.data_ptr(), x.data_ptr(), None, None, 0, dw.data_ptr(), st)

        def ref(x=x, dy=dy, Co=Co, C=C, R=R):
            xs, dys = x[:64].permute(0, 3, 1, 2).float(), dy[:64].permute(0, 3, 1, 2).float()
            return torch.nn.grad.conv2d_weight(xs, (Co, C, R, R), dys, padding=R // 2).permute(0, 2, 3, 1)
        jobs.append((f"wgrad {N}x{H}x{W} {C}->{Co} {R}x{R}", fl, run, dw, (x, dy), d))
    for M, N, K in TN:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        dy = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
        dw = torch.zeros(N, K, device=dev)

        def run(a=a, dy=dy, dw=dw, M=M, N=N, K=K):
            _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dy.data_ptr(), N, a.data_ptr(), K, dw.data_ptr(), st)
        jobs.append((f"gemm_tn {M}x{N}x{K}", 2.0 * M * N * K, run, dw, (a, dy), None))
    res = {}
    for rnd in range(args.rounds):
        for name, fl, run, dw, keep, d in jobs:
            for c in args.cands.split(","):
                if c == "auto":
                    os.environ.pop("ARTSBIR_WGRAD_CFG", None)
                else:
                    os.environ["ARTSBIR_WGRAD_CFG"] = c
                run()
                torch.cuda.synchronize()
                best = 1e30
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    run()
                    e1.record()
                    e1.synchronize()
                    best = min(best, e0.elapsed_time(e1) * 1e3)
                kn = _hip.lib().artsbir_last_kernel().decode()
                r = res.setdefault((name, c), {"us": [], "kn": kn})
                r["us"].append(best)
        print(f"round {rnd}", flush=True)
    os.environ.pop("ARTSBIR_WGRAD_CFG", None)
    for name, fl, *_ in jobs:
        for c in args.cands.split(","):
            r = res[(name, c)]
            us = min(r["us"])
            print(f"{name:36s} cand {c:>4s} {us:9.1f} us {fl / us / 1e6:7.1f} TF  {r['kn']}", flush=True)


if __name__ == "__main__":
    main()
