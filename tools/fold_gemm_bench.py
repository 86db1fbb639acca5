#!/usr/bin/env python3
"""The fold's small per-step GEMMs at the C2 shapes (three BN segments):
artsbir_bn_fold_bwd_prep (the x-side weights W^T diag(b') W, main stream) and
artsbir_bn_fold_wgrad_combine (T = W Gram + the combine, side stream) for every
1x1 conv the backward folds (conv3 and the downsample convs of layers 1-4);
HIP events on the library stream, best of rounds.  ARTSBIR_LIB selects the
library build (A/B of the split-K form: tools/gpu/r6_foldsplit.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

# (Co, Ci): conv3 of layers 1-4, then the downsample convs
SHAPES = [(256, 64), (512, 128), (1024, 256), (2048, 512), (512, 256), (1024, 512), (2048, 1024)]


def timed(f, reps=20, rounds=3):
    best = 1e30
    f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


def main():
    dev = torch.device("cuda:0")
    G = 3
    g = torch.Generator(device=dev).manual_seed(0)
    st = _hip.stream()
    for Co, Ci in SHAPES:
        wt = (torch.randn(Ci, Co, device=dev, generator=g) / Co ** 0.5).bfloat16()
        w = wt.t().contiguous()
        coef = torch.rand(G, 3, Co, device=dev, generator=g)
        prm = torch.rand(G, 4, Co, device=dev, generator=g) + 0.5
        wout = torch.empty(G, Ci, Co + Ci, dtype=torch.bfloat16, device=dev)
        bias = torch.empty(G, Ci, device=dev)
        amat = torch.empty(G, Ci, Co, dtype=torch.bfloat16, device=dev)
        P = torch.randn(G, Co, Ci, device=dev, generator=g)
        gram = torch.randn(G, Ci, Ci, device=dev, generator=g)
        cs = torch.randn(G, 1, Ci, device=dev, generator=g)
        dw = torch.zeros(Co, Ci, device=dev)
        wsp = torch.empty(Co * Ci * (G + 1), device=dev)
        prep = lambda: _hip.call("artsbir_bn_fold_bwd_prep", _hip.DT_BF16, Co, Ci, wt.data_ptr(), coef.data_ptr(),
                                 prm.data_ptr(), 4 * Co, G, wout.data_ptr(), bias.data_ptr(), amat.data_ptr(), st)
        comb = lambda: _hip.call("artsbir_bn_fold_wgrad_combine", _hip.DT_BF16, Co, Ci, G, P.data_ptr(),
                                 gram.data_ptr(), cs.data_ptr(), 1, w.data_ptr(), coef.data_ptr(), prm.data_ptr(),
                                 4 * Co, dw.data_ptr(), wsp.data_ptr(), st)
        tp, tc = timed(prep), timed(comb)
        print(json.dumps({"Co": Co, "Ci": Ci, "prep_us": round(tp, 1), "combine_us": round(tc, 1),
                          "prep_gemm_gflop": round(2.0 * G * Ci * Ci * Co / 1e9, 2)}))


if __name__ == "__main__":
    main()
