#!/usr/bin/env python3
"""Standalone times of the folded BN-backward data gradient (artsbir_conv1x1_dgrad_fold)
on the C2 step's fold shapes, per forced two-operand candidate, next to the
separate weight-gradient operands (artsbir_gemm_tn2 per segment) and the one-pass
form (artsbir_conv1x1_dgrad_fold_wg).  Results are not checked here (see
tests/test_fold_gpu.py); only the time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

# images, H, W, Co (g), Ci (x, dx), fused kind-1 epilogue
SHAPES = [(1152, 56, 56, 256, 64, True), (1152, 56, 56, 256, 64, False), (1152, 28, 28, 512, 128, True),
          (1152, 28, 28, 512, 256, False), (1152, 14, 14, 1024, 256, True), (1152, 7, 7, 2048, 512, True)]


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
    tc = os.path.join(ROOT, "profiles", "tune_r5.txt")
    if os.path.exists(tc):
        _hip.lib().artsbir_tune_load(tc.encode())
    G = 3
    cfgs = os.environ.get("CFGS", "auto,2,10,14,16,17,19,22").split(",")
    for (N, H, W, Co, Ci, fused) in SHAPES:
        M = N * H * W
        g = torch.randn(N, H, W, Co, device=dev).bfloat16()
        x = torch.randn(N, H, W, Ci, device=dev).relu().bfloat16()
        wout = (torch.randn(G, Ci, Co + Ci, device=dev) * 0.05).bfloat16()
        bias = torch.zeros(G, Ci, device=dev)
        dx = torch.empty(N, H, W, Ci, device=dev, dtype=torch.bfloat16)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, Ci, Co, 1, 1, 1, 0)
        desc = None
        if fused:
            y2 = torch.randn(N, H, W, Ci, device=dev).bfloat16()
            bnp = torch.zeros(G, 4, Ci, device=dev)
            bnp[:, 1] = 1.0
            bnp[:, 2] = 1.0
            slots = torch.zeros(G, _hip.NSLOT, 2, Ci, device=dev)
            desc = _hip.BnBwdDesc()
            desc.dtype, desc.kind, desc.pool, desc.ntarget = _hip.DT_BF16, 1, 0, 1
            desc.mask_bn = bnp.data_ptr()
            desc.y[0] = y2.data_ptr()
            desc.mean[0] = bnp.data_ptr()
            desc.istd[0] = bnp[0, 1].data_ptr()
            desc.slots[0] = slots.data_ptr()
            desc.B, desc.H, desc.W, desc.C = N, H, W, Ci
        nb = 2 * M * (Co + Ci + Ci + (Ci if fused else 0))
        print(f"== {N}x{H}x{W} {Co}+{Ci}->{Ci} {'bnb' if fused else 'plain'}: {nb / 1e9:.2f} GB", flush=True)
        for cfg in cfgs:
            if cfg == "auto":
                os.environ.pop("ARTSBIR_PGEMM_CFG", None)
            else:
                os.environ["ARTSBIR_PGEMM_CFG"] = cfg
            try:
                t = timeit(lambda: _hip.call("artsbir_conv1x1_dgrad_fold", d, g.data_ptr(), x.data_ptr(),
                                             wout.data_ptr(), bias.data_ptr(), dx.data_ptr(), desc, G, 4 * Ci, st))
                name = _hip.lib().artsbir_last_kernel().decode()
                print(f"  dgrad cfg {cfg:>4} {name:40s} {t:8.1f} us ({nb / t / 1e3:6.0f} GB/s)", flush=True)
            except _hip.HipError as e:
                print(f"  dgrad cfg {cfg:>4} n/a ({str(e)[:60]})")
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)
        P = torch.zeros(G, Co, Ci, device=dev)
        gram = torch.zeros(G, Ci, Ci, device=dev)
        Ms = M // G

        def tn2():
            for s in range(G):
                _hip.call("artsbir_gemm_tn2", _hip.DT_BF16, Ms, Co, Ci, Ci, g[s * (N // G):].data_ptr(), Co,
                          x[s * (N // G):].data_ptr(), Ci, x[s * (N // G):].data_ptr(), Ci, P[s].data_ptr(),
                          gram[s].data_ptr(), st)
        t = timeit(tn2)
        print(f"  wgrad operands: gemm_tn2 x{G} {_hip.lib().artsbir_last_kernel().decode():26s} {t:8.1f} us", flush=True)
        t = timeit(lambda: _hip.call("artsbir_conv1x1_dgrad_fold_wg", d, g.data_ptr(), x.data_ptr(), wout.data_ptr(),
                                     bias.data_ptr(), dx.data_ptr(), desc, G, 4 * Ci, P.data_ptr(), gram.data_ptr(), st))
        print(f"  one pass: dgrad_fold_wg {_hip.lib().artsbir_last_kernel().decode():32s} {t:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
