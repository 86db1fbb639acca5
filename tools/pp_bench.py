#!/usr/bin/env python3
"""Candidate A/B on the MFMA-bound GEMM / conv shapes of C2 and C5: each forced
pgemm candidate (ARTSBIR_PGEMM_CFG) timed by HIP events on the library stream,
interleaved over rounds in one process (guide §5.4 rule 24), with the max error
against torch.matmul / conv2d on the same bf16 operands.  torch is the checker
and a scale reference only; the product path never calls it.

usage: python tools/pp_bench.py [--cands 0,5,19,22] [--rounds 3] [--only nt|conv]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import _hip  # noqa: E402

NT = [  # M, N, K: C5 projection data gradients (302592 tokens) and forwards, attention-pool k|v
    (302592, 768, 768), (302592, 768, 2304), (302592, 768, 3072), (302592, 2304, 768), (302592, 3072, 768),
    (57600, 4096, 2048),
]
CONV = [  # N, H, W, C, Cout, R (3x3 stride 1 pad 1 forwards of C2 at 1152 images)
    (1152, 56, 56, 64, 64, 3), (1152, 28, 28, 128, 128, 3), (1152, 14, 14, 256, 256, 3), (1152, 7, 7, 512, 512, 3),
    (1152, 56, 56, 64, 256, 1), (1152, 28, 28, 512, 128, 1),
    (1152, 28, 28, 128, 512, 1), (1152, 14, 14, 256, 1024, 1), (1152, 7, 7, 512, 2048, 1),  # bottleneck conv3
    (1152, 112, 112, 32, 64, 3), (1152, 112, 112, 32, 32, 3), (1152, 112, 112, 64, 32, 3),  # stem (and its dgrads)
]


def ev_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best * 1e3


def set_cfg(c):
    if c == "auto":
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)
    else:
        os.environ["ARTSBIR_PGEMM_CFG"] = c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cands", default="0,5,19,22")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    cands = args.cands.split(",")
    dev = torch.device("cuda:0")
    st = _hip.stream()  # the library's default stream is torch's current stream
    torch.manual_seed(0)
    jobs = []
    if args.only in ("", "nt"):
        for M, N, K in NT:
            a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            b = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ref = torch.matmul(a, b.t()).float()

            def run(a=a, b=b, c=c, M=M, N=N, K=K):
                _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, a.data_ptr(), K, b.data_ptr(), c.data_ptr(), N, 0, 0,
                          None, None, st)
            jobs.append((f"nt {M}x{N}x{K}", 2.0 * M * N * K, run, c, ref, (a, b)))
    if args.only in ("", "conv"):
        for N, H, W, C, Co, R in CONV:
            x = (torch.rand(N, H, W, C, device=dev) * 2 - 1).bfloat16()
            w = ((torch.rand(Co, R, R, C, device=dev) * 2 - 1) / (C * R * R) ** 0.5).bfloat16()
            y = torch.empty(N * H * W, Co, device=dev, dtype=torch.bfloat16)
            stats = torch.zeros(_hip.NSLOT, 2, Co, device=dev)
            ref = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=R // 2).permute(0, 2, 3, 1)
            ref = ref.reshape(-1, Co).float()
            d = _hip.conv_desc(torch.bfloat16, N, H, W, C, Co, R, R, 1, R // 2)

            def run(x=x, w=w, y=y, d=d, Co=Co, stats=stats):
                _hip.call("artsbir_conv2d_fwd", d, x.data_ptr(), w.data_ptr(), y.data_ptr(), Co, 0, 0, None, None,
                          None, 0, stats.data_ptr(), st)
            jobs.append((f"conv {N}x{H}x{W} {C}->{Co} {R}x{R}", 2.0 * N * H * W * Co * C * R * R, run, y, ref,
                         (x, w, stats)))
    res = {}
    for rnd in range(args.rounds):
        for name, fl, run, out, ref, _keep in jobs:
            for c in cands:
                set_cfg(c)
                out.fill_(float("nan"))
                us = ev_time(run)
                kn = _hip.lib().artsbir_last_kernel().decode()
                err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                r = res.setdefault((name, c), {"us": [], "kn": kn, "err": err, "fl": fl})
                r["us"].append(us)
                r["err"] = max(r["err"], err)
        print(f"round {rnd} done", flush=True)
    set_cfg("auto")
    for name, fl, *_ in jobs:
        for c in cands:
            r = res[(name, c)]
            us = sorted(r["us"])
            print(f"{name:34s} cand {c:>3s} {us[0]:9.1f} us (med {us[len(us) // 2]:9.1f}) "
                  f"{fl / us[0] / 1e6:7.1f} TF  relerr {r['err']:.2e}  {r['kn']}", flush=True)


if __name__ == "__main__":
    main()
