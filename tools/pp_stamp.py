#!/usr/bin/env python3
"""Segment shares of the pp256 K-tile loop from the PP_STAMP=1 diagnostic build
(art-sbir_amd/build_var/libartsbir_stamp.so, ARTSBIR_LIB): per wave group, the
cycles each segment takes as a share of the loop, on one GEMM shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("ARTSBIR_LIB", os.path.join(ROOT, "art-sbir_amd", "build_var", "libartsbir_stamp.so"))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
import torch  # noqa: E402

import _hip  # noqa: E402

SEG = ["loop", "px issue", "ds_read a", "barrier1", "mfma a", "barrier2", "ch issue", "vmcnt", "ds_read b",
       "barrier3", "mfma b", "barrier4", "epilogue"]


def main():
    M, N, K = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (302592, 768, 2304))]
    dev = torch.device("cuda:0")
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    b = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for cand in ("22", "23"):
        ts = torch.zeros(8192 * 8 * 16, dtype=torch.int64, device=dev)
        os.environ["ARTSBIR_PP_TS"] = str(ts.data_ptr())
        os.environ["ARTSBIR_PGEMM_CFG"] = cand
        _hip.call("artsbir_gemm_nt", _hip.DT_BF16, M, N, K, a.data_ptr(), K, b.data_ptr(), c.data_ptr(), N, 0, 0,
                  None, None, _hip.stream())
        torch.cuda.synchronize()
        print(cand, _hip.lib().artsbir_last_kernel().decode())
        t = ts.view(-1, 8, 16).cpu().double()
        live = t[:, :, 13] > 0
        for g, ws in (("group0", slice(0, 4)), ("group1", slice(4, 8))):
            sel = t[:, ws][live[:, ws]]
            tot = sel[:, :13].sum()
            ktiles = sel[:, 13].sum()
            print(f"  {g}: {sel.shape[0]} waves, {tot / ktiles:8.0f} cycles per K-tile")
            for k, nm in enumerate(SEG):
                print(f"    {nm:10s} {100 * sel[:, k].sum() / tot:6.2f} %  {sel[:, k].sum() / ktiles:8.1f} cyc/K-tile")


if __name__ == "__main__":
    main()
