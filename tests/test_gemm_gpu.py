"""Implicit-GEMM conv / dense GEMM / weight-gradient kernels vs torch fp32 (CPU) references."""
import pytest
import torch
import torch.nn.functional as F

import _hip

pytestmark = pytest.mark.gpu

CASES = [
    # N, H, W, C, Cout, R, S, stride, pad
    (2, 9, 7, 8, 32, 3, 3, 2, 1),
    (2, 8, 8, 32, 64, 3, 3, 1, 1),
    (3, 7, 5, 64, 256, 1, 1, 1, 0),
    (2, 14, 14, 128, 128, 3, 3, 1, 1),
    (1, 5, 5, 256, 72, 1, 1, 1, 0),
]


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_fwd(case, dt, dev):
    N, H, W, C, Co, R, S, st, pd = case
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Co, C, R, S, generator=g) / (C * R * S) ** 0.5
    sc = torch.rand(C, generator=g) + 0.5
    sh = torch.randn(C, generator=g) * 0.1
    if dt == torch.bfloat16:
        x = x.bfloat16().float(); w = w.bfloat16().float()
    act = torch.relu(x * sc[None, :, None, None] + sh[None, :, None, None])
    if dt == torch.bfloat16:
        act = act.bfloat16().float()
    ref = F.conv2d(act, w, stride=st, padding=pd)
    Ho, Wo = ref.shape[2:]
    xd = _nhwc(x).to(dev, dt)
    wd = w.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    y = torch.empty(N * Ho * Wo, Co, device=dev, dtype=torch.float32)
    stats = torch.zeros(_hip.NSLOT, 2, Co, device=dev)
    d = _hip.conv_desc(dt, N, H, W, C, Co, R, S, st, pd)
    scd, shd = sc.to(dev), sh.to(dev)  # keep device copies alive across the call
    _hip.call("artsbir_conv2d_fwd", d, xd.data_ptr(), wd.data_ptr(), y.data_ptr(), Co, 1, 0, None,
              scd.data_ptr(), shd.data_ptr(), 1, stats.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    out = y.cpu().view(N, Ho, Wo, Co).permute(0, 3, 1, 2)
    tol = 1e-4 if dt == torch.float32 else 2e-3
    assert torch.allclose(out, ref, atol=tol, rtol=tol), (out - ref).abs().max()
    s = stats.sum(0).cpu()
    r2 = ref.permute(0, 2, 3, 1).reshape(-1, Co)
    assert torch.allclose(s[0], r2.sum(0), atol=1e-2, rtol=1e-3)
    assert torch.allclose(s[1], (r2 * r2).sum(0), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_wgrad(case, dt, dev):
    N, H, W, C, Co, R, S, st, pd = case
    if Co % 8:
        pytest.skip()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Co, C, R, S, generator=g)
    Ho = (H + 2 * pd - R) // st + 1
    Wo = (W + 2 * pd - S) // st + 1
    dy = torch.randn(N, Co, Ho, Wo, generator=g)
    if dt == torch.bfloat16:
        x = x.bfloat16().float(); dy = dy.bfloat16().float()
    xr = x.clone().requires_grad_(False)
    wr = w.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=st, padding=pd).backward(dy)
    ref = wr.grad.permute(0, 2, 3, 1).contiguous()  # KRSC
    dw = torch.zeros(Co, R, S, C, device=dev)
    d = _hip.conv_desc(dt, N, H, W, C, Co, R, S, st, pd)
    dyd, xd = _nhwc(dy).to(dev, dt), _nhwc(x).to(dev, dt)
    _hip.call("artsbir_conv2d_wgrad", d, dyd.data_ptr(), xd.data_ptr(),
              None, None, 0, dw.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    tol = 1e-3 if dt == torch.float32 else 2e-2
    assert torch.allclose(dw.cpu(), ref, atol=tol, rtol=tol), (dw.cpu() - ref).abs().max()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(100, 96, 64), (37, 512, 2048), (300, 40, 24)])
def test_gemm_nt_tn(dt, M, N, K, dev):
    g = torch.Generator().manual_seed(2)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    if dt == torch.bfloat16:
        a = a.bfloat16().float(); b = b.bfloat16().float()
    ref = a @ b.T + bias
    c = torch.empty(M, N, device=dev)
    ad, bd, biasd = a.to(dev, dt), b.to(dev, dt), bias.to(dev)
    _hip.call("artsbir_gemm_nt", _hip.dtype_code(dt), M, N, K, ad.data_ptr(), K,
              bd.data_ptr(), c.data_ptr(), N, 1, 0, biasd.data_ptr(), None, _hip.stream())
    torch.cuda.synchronize()
    tol = 1e-3 if dt == torch.float32 else 1e-2
    assert torch.allclose(c.cpu(), ref, atol=tol * K ** 0.5, rtol=tol)
    # dw[N][K] = dy^T x
    dy = torch.randn(M, N, generator=g)
    if dt == torch.bfloat16:
        dy = dy.bfloat16().float()
    dw = torch.zeros(N, K, device=dev)
    dyd = dy.to(dev, dt)
    _hip.call("artsbir_gemm_tn", _hip.dtype_code(dt), M, N, K, dyd.data_ptr(), N,
              ad.data_ptr(), K, dw.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    ref2 = dy.T @ a
    assert torch.allclose(dw.cpu(), ref2, atol=tol * M ** 0.5, rtol=tol)
