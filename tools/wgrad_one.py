#!/usr/bin/env python3
"""One weight-gradient shape of tools/wgrad_bench.py, one forced candidate, a few
launches (for rocprofv3 --pmc passes):  wgrad_one.py conv|dense <index> <cfg>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "art-sbir_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import _hip  # noqa: E402
import wgrad_bench as wb  # noqa: E402

kind, idx, cfg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
os.environ["ARTSBIR_WGRAD_CFG"] = cfg
dev = torch.device("cuda:0")
st = _hip.stream()
if kind == "conv":
    H, W, C, Co, R, s = wb.CONV[idx]
    B = wb.B
    x = torch.randn(B, H, W, C, device=dev).bfloat16()
    dy = torch.randn(B * (H // s) * (W // s), Co, device=dev).bfloat16()
    dw = torch.zeros(Co, R * R * C, device=dev)
    d = _hip.conv_desc(torch.bfloat16, B, H, W, C, Co, R, R, s, R // 2)
    run = lambda: _hip.call("artsbir_conv2d_wgrad", d, dy.data_ptr(), x.data_ptr(), None, None, 0, dw.data_ptr(), st)  # noqa: E731
else:
    M, N, K = wb.DENSE[idx]
    dy = torch.randn(M, N, device=dev).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    dw = torch.zeros(N, K, device=dev)
    run = lambda: _hip.call("artsbir_gemm_tn", _hip.DT_BF16, M, N, K, dy.data_ptr(), N, x.data_ptr(), K,  # noqa: E731
                            dw.data_ptr(), st)
for _ in range(5):
    run()
torch.cuda.synchronize()
print(_hip.lib().artsbir_last_kernel().decode())
