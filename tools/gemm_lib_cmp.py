#!/usr/bin/env python3
"""C5 projection GEMM shapes (302592 tokens = 512 triplets x 3 x 197): the
library's hand-written bf16 GEMMs (artsbir_gemm_nt: c = a b^T; artsbir_gemm_tn:
dw += dy^T x, f32) next to torch.matmul (hipBLASLt) on the same operands, for
scale only (the product path does not call torch.matmul)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))

import torch  # noqa: E402

import _hip  # noqa: E402

M = 302592
NT = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]  # N (out), K (in)


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
    for N, K in NT:
        a = torch.randn(M, K, device=dev).bfloat16()
        b = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t_own = timeit(lambda: _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, a.data_ptr(), K, b.data_ptr(),
                                         c.data_ptr(), N, 0, 0, None, None, st))
        kn = _hip.lib().artsbir_last_kernel().decode()
        t_lib = timeit(lambda: torch.matmul(a, b.t(), out=c))
        print(f"NT M={M} N={N} K={K}: own {t_own:7.1f} us {fl / t_own / 1e6:6.1f} TF ({kn}) | "
              f"torch.matmul {t_lib:7.1f} us {fl / t_lib / 1e6:6.1f} TF", flush=True)
        dy = torch.randn(M, N, device=dev).bfloat16()
        dw = torch.zeros(N, K, device=dev)
        dwb = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        t_own = timeit(lambda: _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dy.data_ptr(), N, a.data_ptr(), K,
                                         dw.data_ptr(), st))
        kn = _hip.lib().artsbir_last_kernel().decode()
        t_lib = timeit(lambda: torch.matmul(dy.t(), a, out=dwb))
        print(f"TN M={M} N={N} K={K}: own {t_own:7.1f} us {fl / t_own / 1e6:6.1f} TF ({kn}) | "
              f"torch.matmul {t_lib:7.1f} us {fl / t_lib / 1e6:6.1f} TF", flush=True)
        del a, b, c, dy, dw, dwb


if __name__ == "__main__":
    main()
