#!/usr/bin/env python3
"""The ViT MLP backward's c_proj data gradient at C5 size (M = 302592 tokens,
N = 3072, K = 768): artsbir_gemm_nt_gate (QuickGELU-gated epilogue with the
column-sum slots) against the same call without the slots and against the plain
artsbir_gemm_nt, HIP events on the library stream, best of rounds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M, N, K = 302592, 3072, 768
    g = torch.Generator(device=dev).manual_seed(0)
    a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
    x = (torch.rand(M, N, device=dev, generator=g) * 6 - 3).bfloat16()
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    slots = torch.zeros(_hip.NSLOT, 2, N, device=dev)
    st = _hip.stream()
    runs = {
        "gate+sums": lambda: _hip.call("artsbir_gemm_nt_gate", M, N, K, a.data_ptr(), K, w.data_ptr(), c.data_ptr(),
                                       N, x.data_ptr(), slots.data_ptr(), st),
        "gate": lambda: _hip.call("artsbir_gemm_nt_gate", M, N, K, a.data_ptr(), K, w.data_ptr(), c.data_ptr(), N,
                                  x.data_ptr(), None, st),
        "plain": lambda: _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, a.data_ptr(), K, w.data_ptr(),
                                   c.data_ptr(), N, 0, 0, None, None, st),
        "plain+sums": lambda: _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, a.data_ptr(), K, w.data_ptr(),
                                        c.data_ptr(), N, 0, 0, None, slots.data_ptr(), st),
    }
    best = {k: 1e30 for k in runs}
    for k, f in runs.items():
        f()
    torch.cuda.synchronize()
    for _ in range(3):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(torch.cuda.current_stream())
            for _ in range(5):
                f()
            e1.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            best[k] = min(best[k], e0.elapsed_time(e1) / 5)
    for k, v in best.items():
        print(json.dumps({"run": k, "ms": round(v, 4), "TFLOPs": round(2.0 * M * N * K / v / 1e9, 1)}))


if __name__ == "__main__":
    main()
