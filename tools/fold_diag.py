"""Diagnostic: artsbir_conv1x1_dgrad_fold on one forced candidate over shapes,
with each operand zeroed in turn, vs float64 (which part of [g | x] w^T + bias
goes wrong).  python tools/fold_diag.py <cfg>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "art-sbir_amd")]
import torch  # noqa: E402

import _hip  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "22"
dev = torch.device("cuda:0")
torch.manual_seed(0)
for (N, H, W, Co, Ci) in [(2, 14, 14, 256, 512), (2, 16, 16, 256, 512), (2, 14, 14, 512, 256), (2, 16, 16, 256, 256),
                          (2, 16, 16, 512, 512), (2, 16, 16, 256, 768), (4, 16, 16, 1024, 512)]:
    M = N * H * W
    K = Co + Ci
    g = torch.randn(M, Co).bfloat16()
    x = torch.randn(M, Ci).bfloat16()
    w = (torch.randn(Ci, K) / K ** 0.5).bfloat16()
    b = torch.randn(Ci)
    for part in ("all", "g_only", "x_only", "bias_only"):
        gg = g if part in ("all", "g_only") else torch.zeros_like(g)
        xx = x if part in ("all", "x_only") else torch.zeros_like(x)
        bb = b if part in ("all", "bias_only") else torch.zeros_like(b)
        ref = torch.cat([gg, xx], 1).double() @ w.double().T + bb.double()
        gd, xd, wd, bd = gg.to(dev), xx.to(dev), w.to(dev), bb.to(dev)
        dx = torch.full((M, Ci), float("nan"), dtype=torch.bfloat16, device=dev)
        d = _hip.conv_desc(torch.bfloat16, N, H, W, Ci, Co, 1, 1, 1, 0)
        os.environ["ARTSBIR_PGEMM_CFG"] = cfg
        _hip.call("artsbir_conv1x1_dgrad_fold", d, gd.data_ptr(), xd.data_ptr(), wd.data_ptr(), bd.data_ptr(),
                  dx.data_ptr(), None, 1, 4 * Ci, _hip.stream())
        torch.cuda.synchronize()
        name = _hip.lib().artsbir_last_kernel().decode()
        out = dx.double().cpu()
        err = ((out - ref).norm() / ref.norm().clamp_min(1e-30)).item()
        bad = ((out - ref).abs() > 0.05 * ref.abs().max()).nonzero()
        rows = sorted(set(bad[:, 0].tolist()))
        cols = sorted(set(bad[:, 1].tolist()))
        print(f"M={M} Co={Co} Ci={Ci} {part:9s} {name:28s} rel {err:.2e}  bad rows {len(rows)} "
              f"[{rows[:3]}..{rows[-3:]}] cols {len(cols)} [{cols[:3]}..{cols[-3:]}]", flush=True)
