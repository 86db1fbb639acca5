"""Transformer block of models.py:382-417 (forward parity).

CPU: the oracle restatement against the PyTorch modules the reference's block
is made of (nn.MultiheadAttention, nn.LayerNorm in fp32, Linear) — the
reference's arithmetic lives in PyTorch, so this pins the restatement.
GPU: the HIP forward (artsbir_layernorm_fwd, gemm_nt, artsbir_mha_fwd,
artsbir_quickgelu) against the oracle, f32 within 2e-4 relative, bf16 within
3e-2."""
import pytest
import torch
from torch import nn

from oracle import encoder as oenc


def _torch_block(E, heads, seed):
    torch.manual_seed(seed)
    attn = nn.MultiheadAttention(E, heads)
    ln1, ln2 = nn.LayerNorm(E), nn.LayerNorm(E)
    fc, proj = nn.Linear(E, 4 * E), nn.Linear(4 * E, E)
    for m in (ln1, ln2):  # non-trivial affine
        nn.init.normal_(m.weight, 1.0, 0.1)
        nn.init.normal_(m.bias, 0.0, 0.1)
    sd = {"attn.in_proj_weight": attn.in_proj_weight, "attn.in_proj_bias": attn.in_proj_bias,
          "attn.out_proj.weight": attn.out_proj.weight, "attn.out_proj.bias": attn.out_proj.bias,
          "ln_1.weight": ln1.weight, "ln_1.bias": ln1.bias, "ln_2.weight": ln2.weight, "ln_2.bias": ln2.bias,
          "mlp.c_fc.weight": fc.weight, "mlp.c_fc.bias": fc.bias,
          "mlp.c_proj.weight": proj.weight, "mlp.c_proj.bias": proj.bias}
    sd = {k: v.detach() for k, v in sd.items()}

    def run(x, mask=None):
        h = ln1(x.float()).to(x.dtype)
        x = x + attn(h, h, h, need_weights=False, attn_mask=mask)[0]
        h = ln2(x.float()).to(x.dtype)
        f = fc(h)
        return x + proj(f * torch.sigmoid(1.702 * f))
    return sd, run


@pytest.mark.parametrize("masked", [False, True])
def test_oracle_block_matches_torch_modules(masked):
    E, heads, L, N = 128, 2, 9, 3
    sd, run = _torch_block(E, heads, 5)
    x = torch.randn(L, N, E, generator=torch.Generator().manual_seed(6))
    mask = torch.triu(torch.full((L, L), float("-inf")), 1) if masked else None
    with torch.no_grad():
        ref = run(x, mask)
    got = oenc.residual_attention_block(x, sd, heads, mask)
    assert torch.allclose(got, ref, atol=2e-5, rtol=1e-5), (got - ref).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("L,N,E,heads,masked", [(9, 3, 128, 2, False), (197, 2, 768, 12, False),
                                                 (17, 4, 256, 4, True)])
def test_hip_block_matches_oracle(L, N, E, heads, masked, dtype, tol, dev):
    import models
    torch.manual_seed(11)
    mask = torch.triu(torch.full((L, L), float("-inf")), 1) if masked else None
    blk = models.ResidualAttentionBlock(E, heads, attn_mask=mask)
    for m in (blk.ln_1, blk.ln_2):
        nn.init.normal_(m.weight, 1.0, 0.1)
        nn.init.normal_(m.bias, 0.0, 0.1)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    x = torch.randn(L, N, E, generator=torch.Generator().manual_seed(12))
    if dtype == torch.bfloat16:
        x = x.bfloat16().float()
    ref = oenc.residual_attention_block(x.double(), {k: v.double() for k, v in sd.items()}, heads,
                                        mask.double() if mask is not None else None)
    blk = blk.to(dev)
    got = blk(x.to(dev, dtype)).float().cpu()
    err = (got.double() - ref).norm() / ref.norm()
    assert err < tol, float(err)


def _block_oracle_grads(blk_sd, x, heads, mask, w):
    """f64 oracle forward + autograd backward of sum(y * w)"""
    sd = {k: v.double().clone().requires_grad_(True) for k, v in blk_sd.items()}
    xr = x.double().clone().requires_grad_(True)
    y = oenc.residual_attention_block(xr, sd, heads, mask.double() if mask is not None else None)
    (y * w).sum().backward()
    return y.detach(), xr.grad, {k: v.grad for k, v in sd.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 4e-2)])
@pytest.mark.parametrize("L,N,E,heads,masked", [(9, 3, 128, 2, False), (197, 2, 768, 12, False),
                                                 (17, 4, 256, 4, True)])
def test_hip_block_backward_matches_oracle(L, N, E, heads, masked, dtype, tol, dev):
    """input and parameter gradients of the block (artsbir_mha_bwd, layernorm_bwd,
    quickgelu_bwd, the projection GEMMs) against float64 autograd of the oracle"""
    import models
    torch.manual_seed(13)
    mask = torch.triu(torch.full((L, L), float("-inf")), 1) if masked else None
    blk = models.ResidualAttentionBlock(E, heads, attn_mask=mask)
    for m in (blk.ln_1, blk.ln_2):
        nn.init.normal_(m.weight, 1.0, 0.1)
        nn.init.normal_(m.bias, 0.0, 0.1)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    x = torch.randn(L, N, E, generator=torch.Generator().manual_seed(14))
    if dtype == torch.bfloat16:
        x = x.bfloat16().float()
    w = torch.randn(L, N, E, generator=torch.Generator().manual_seed(15), dtype=torch.float64)
    y_ref, dx_ref, g_ref = _block_oracle_grads(sd, x, heads, mask, w)
    blk = blk.to(dev)
    xm = x.to(dev, dtype).requires_grad_(True)
    y = blk(xm)
    (y.float() * w.float().to(dev)).sum().backward()
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y.detach(), y_ref) < tol
    assert rel(xm.grad, dx_ref) < tol * 2, rel(xm.grad, dx_ref)
    named = dict(blk.named_parameters())
    for k, g in g_ref.items():
        e = rel(named[k].grad, g)
        assert e < tol * 5, (k, e)


@pytest.mark.gpu
def test_fp8_gemm_matches_dequantized_reference(dev):
    """artsbir_quantize_fp8 = torch's e4m3fn cast of x / (amax / 448) bit for bit;
    artsbir_gemm_nt_fp8 = the f64 product of the dequantized operands (+ bias),
    within f32 accumulation error; ragged M / N tiles"""
    import _hip
    import vit
    g = torch.Generator(device=dev).manual_seed(3)
    # (600, 520, 384), (256, 768, 3072): the 256 x 256 LDS-DMA kernel with ragged tiles and a long K
    for M, N, K in [(200, 136, 256), (130, 2304, 768), (1, 1, 128), (600, 520, 384), (256, 768, 3072)]:
        a = torch.randn(M, K, device=dev, generator=g)
        b = torch.randn(N, K, device=dev, generator=g) * 0.05
        bias = torch.randn(N, device=dev, generator=g)
        qa, sa = vit._fp8(a)
        qb, sb = vit._fp8(b)
        for t, q, s in ((a, qa, sa), (b, qb, sb)):
            tc = t.cpu()  # the oracle on the CPU: IEEE f32 division, then torch's RNE e4m3fn cast
            v = tc / (tc.abs().max() / 448.0)
            want = v.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
            bad = (q != want).nonzero()
            if len(bad):
                i = tuple(bad[0].tolist())
                print("fp8 mismatch", len(bad), "of", q.numel(), "value", v[i].item(), "mine", q[i].item(),
                      "torch", want[i].item())
            assert torch.equal(q, want)
            assert torch.allclose(s, t.abs().max().reshape(1) / 448.0, rtol=1e-7)
        out = torch.empty(M, N, device=dev)
        _hip.call("artsbir_gemm_nt_fp8", M, N, K, qa.data_ptr(), qb.data_ptr(), sa.data_ptr(), sb.data_ptr(),
                  bias.data_ptr(), out.data_ptr(), _hip.DT_F32, 0, _hip.stream())
        da = qa.view(torch.float8_e4m3fn).double().cpu() * sa.double().cpu()
        db = qb.view(torch.float8_e4m3fn).double().cpu() * sb.double().cpu()
        ref = da @ db.T + bias.double().cpu()
        err = (out.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 5e-5, (M, N, K, err)  # f32 accumulation of up to 3072 products
        # accumulate = 1 onto an f32 output (the residual stream)
        init = torch.randn(M, N, device=dev, generator=g)
        out2 = init.clone()
        _hip.call("artsbir_gemm_nt_fp8", M, N, K, qa.data_ptr(), qb.data_ptr(), sa.data_ptr(), sb.data_ptr(),
                  bias.data_ptr(), out2.data_ptr(), _hip.DT_F32, 1, _hip.stream())
        err2 = (out2.double().cpu() - init.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err2 < 5e-5, (M, N, K, err2)


def _vit_pair(seed, res=64, patch=16, width=128, layers=2, heads=2, out=64):
    import models
    torch.manual_seed(seed)
    m = models.VisionTransformer(res, patch, width, layers, heads, out)
    for blk in m.transformer.resblocks:
        for ln in (blk.ln_1, blk.ln_2):
            nn.init.normal_(ln.weight, 1.0, 0.1)
            nn.init.normal_(ln.bias, 0.0, 0.1)
    return m, {k: v.detach().clone() for k, v in m.state_dict().items()}


@pytest.mark.gpu
@pytest.mark.parametrize("mode,tol", [("f32", 3e-4), ("bf16", 5e-2), ("fp8", 1.5e-1)])
def test_vit_encoder_matches_oracle(mode, tol, dev):
    """the ViT encoder (patch GEMM, tokens, ln_pre, blocks, ln_post, proj) forward and
    its gradients (fp8: forward GEMMs in e4m3, backward bf16) vs float64 autograd"""
    m, sd = _vit_pair(21)
    x = torch.randn(3, 3, 64, 64, generator=torch.Generator().manual_seed(22))
    w = torch.randn(3, 64, generator=torch.Generator().manual_seed(23), dtype=torch.float64)
    sdr = {k: v.double().clone().requires_grad_(True) for k, v in sd.items()}
    y_ref = oenc.vision_transformer(x.double(), sdr, 16, 2)
    (y_ref * w).sum().backward()
    m = m.to(dev)
    m.compute_dtype = {"f32": torch.float32, "bf16": torch.bfloat16, "fp8": "fp8"}[mode]
    y = m(x.to(dev))
    assert y.dtype == torch.float32 and y.shape == (3, 64)
    (y * w.float().to(dev)).sum().backward()
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y.detach(), y_ref.detach()) < tol, rel(y.detach(), y_ref.detach())
    named = dict(m.named_parameters())
    worst = max((rel(named[k].grad, v.grad), k) for k, v in sdr.items())
    assert worst[0] < tol * 5, worst


@pytest.mark.gpu
def test_vit_backward_kernels_individually(dev):
    """artsbir_layernorm_bwd, artsbir_quickgelu_bwd and artsbir_mha_bwd each
    against float64 autograd of their oracle op (f32 storage)"""
    import _hip
    g = torch.Generator().manual_seed(31)
    st = _hip.stream()
    # LayerNorm
    rows, C = 37, 768
    x = torch.randn(rows, C, generator=g)
    gam, bet = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g)
    res = torch.randn(rows, C, generator=g)
    xr = x.double().requires_grad_(True)
    gr, br = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    (oenc.layernorm_fp32(xr, gr, br) * dy.double()).sum().backward()
    X, G, Dy, Rs = (t.to(dev) for t in (x, gam, dy, res))
    dx = torch.empty_like(X)
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    _hip.call("artsbir_layernorm_bwd", _hip.DT_F32, X.data_ptr(), G.data_ptr(), Dy.data_ptr(), rows, C, 1e-5,
              Rs.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), st)
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(dx, xr.grad + res.double()) < 1e-5
    assert rel(dg, gr.grad) < 1e-5 and rel(db, br.grad) < 1e-5
    # QuickGELU
    v = torch.randn(1000, generator=g) * 3
    vr = v.double().requires_grad_(True)
    gv = torch.randn(1000, generator=g)
    (oenc.quick_gelu(vr) * gv.double()).sum().backward()
    V, GV = v.to(dev), gv.to(dev)
    dv = torch.empty_like(V)
    _hip.call("artsbir_quickgelu_bwd", _hip.DT_F32, V.data_ptr(), GV.data_ptr(), 1000, dv.data_ptr(), st)
    assert rel(dv, vr.grad) < 1e-5
    # attention core
    L, N, heads = 9, 3, 2
    E = 64 * heads
    qkv = torch.randn(L * N, 3 * E, generator=g)
    dO = torch.randn(L * N, E, generator=g)
    qr = qkv.double().requires_grad_(True)
    q, k, vv = qr.view(L, N, 3 * E).split(E, dim=-1)

    def hd(t):
        return t.reshape(L, N, heads, 64).permute(1, 2, 0, 3)
    p = torch.softmax((hd(q) / 8.0) @ hd(k).transpose(-1, -2), dim=-1)
    o = (p @ hd(vv)).permute(2, 0, 1, 3).reshape(L * N, E)
    (o * dO.double()).sum().backward()
    Q, DO = qkv.to(dev), dO.to(dev)
    out = torch.empty(L * N, E, device=dev)
    lse = torch.empty(L * N * heads, device=dev)
    _hip.call("artsbir_mha_fwd_lse", _hip.DT_F32, Q.data_ptr(), L, N, heads, None, out.data_ptr(), lse.data_ptr(), st)
    assert rel(out, o.detach()) < 1e-5
    dq = torch.empty_like(Q)
    dsc = torch.empty(L * N * heads, device=dev)
    _hip.call("artsbir_mha_bwd", _hip.DT_F32, Q.data_ptr(), out.data_ptr(), DO.data_ptr(), lse.data_ptr(), L, N,
              heads, None, dq.data_ptr(), dsc.data_ptr(), st)
    for part, sl in (("q", slice(0, E)), ("k", slice(E, 2 * E)), ("v", slice(2 * E, 3 * E))):
        assert rel(dq[:, sl], qr.grad[:, sl]) < 1e-5, part


@pytest.mark.gpu
@pytest.mark.parametrize("L,N,heads,masked", [(1, 2, 1, False), (9, 3, 2, True), (32, 2, 2, False),
                                              (33, 2, 3, True), (197, 4, 12, False), (197, 2, 2, True),
                                              (256, 2, 2, False), (100, 3, 4, False), (160, 2, 2, True),
                                              (64, 5, 1, False)])
def test_mfma_attention_bf16(L, N, heads, masked, dev):
    """the bf16 attention core (attn.hip: MFMA forward with online softmax, the
    one-workgroup query- and key-side MFMA backward, both LDS-DMA staged, one
    instantiation per count of 32-row blocks) against float64 autograd on the same bf16 inputs:
    output and gradients within 2e-2 relative L2 (bf16 P / dS operands and bf16
    outputs), log-sum-exp within 1e-4"""
    import _hip
    g = torch.Generator().manual_seed(1000 + L)
    st = _hip.stream()
    E = 64 * heads
    qkv = torch.randn(L * N, 3 * E, generator=g).bfloat16()
    dO = torch.randn(L * N, E, generator=g).bfloat16()
    mask = None
    if masked:  # causal -inf plus finite noise (an arbitrary float attn_mask)
        mask = torch.full((L, L), float("-inf")).triu(1) + 0.5 * torch.randn(L, L, generator=g)
        mask = mask.bfloat16().float()  # the block casts the mask to x.dtype
    qr = qkv.double().requires_grad_(True)
    q, k, vv = qr.view(L, N, 3 * E).split(E, dim=-1)

    def hd(t):
        return t.reshape(L, N, heads, 64).permute(1, 2, 0, 3)
    s = (hd(q) / 8.0) @ hd(k).transpose(-1, -2)
    if mask is not None:
        s = s + mask.double()
    lse_ref = torch.logsumexp(s, dim=-1)  # [N, heads, L]
    p = torch.softmax(s, dim=-1)
    o = (p @ hd(vv)).permute(2, 0, 1, 3).reshape(L * N, E)
    (o * dO.double()).sum().backward()
    Q, DO = qkv.to(dev), dO.to(dev)
    M = mask.to(dev) if mask is not None else None
    out = torch.empty(L * N, E, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(L * N * heads, device=dev)
    _hip.call("artsbir_mha_fwd_lse", _hip.DT_BF16, Q.data_ptr(), L, N, heads, M.data_ptr() if M is not None else None,
              out.data_ptr(), lse.data_ptr(), st)
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(out, o.detach()) < 2e-2, rel(out, o.detach())
    lse_got = lse.view(L, N, heads).permute(1, 2, 0).double().cpu()
    assert (lse_got - lse_ref.detach()).abs().max().item() < 1e-4
    dq = torch.empty_like(Q)
    dsc = torch.empty(L * N * heads, device=dev)
    _hip.call("artsbir_mha_bwd", _hip.DT_BF16, Q.data_ptr(), out.data_ptr(), DO.data_ptr(), lse.data_ptr(), L, N,
              heads, M.data_ptr() if M is not None else None, dq.data_ptr(), dsc.data_ptr(), st)
    for part, sl in (("q", slice(0, E)), ("k", slice(E, 2 * E)), ("v", slice(2 * E, 3 * E))):
        ref = qr.grad[:, sl]
        if ref.norm() == 0:  # L = 1: dq = dk = 0 up to the rounding of D = dO . O
            assert dq[:, sl].abs().max().item() < 1e-3, part
        else:
            assert rel(dq[:, sl], ref) < 2e-2, (part, rel(dq[:, sl], ref))


@pytest.mark.gpu
def test_fused_amax_producers_quantise_identically(dev):
    """the fp8 producers with the fused amax (LayerNorm, QuickGELU, attention) give
    exactly the codes and scale of the separate amax pass over their outputs"""
    import _hip
    import vit
    g = torch.Generator(device=dev).manual_seed(17)
    st = _hip.stream()
    rows, C = 1000, 768
    x = torch.randn(rows, C, device=dev, generator=g).bfloat16()
    w = 1 + 0.1 * torch.randn(C, device=dev, generator=g)
    b = 0.1 * torch.randn(C, device=dev, generator=g)
    pm = vit._pmax(dev)
    y = vit._ln(x, w, b, 1e-5, pm)
    for t, p in ((y, pm),):
        q0, s0 = vit._fp8(t)
        q1, s1 = vit._fp8(t, p)
        assert torch.equal(q0, q1) and torch.equal(s0, s1)
    f = torch.randn(rows, 3072, device=dev, generator=g).bfloat16() * 3
    a = torch.empty_like(f)
    pm = vit._pmax(dev)
    _hip.call("artsbir_quickgelu_pmax", _hip.DT_BF16, f.data_ptr(), f.numel(), a.data_ptr(), pm.data_ptr(), st)
    q0, s0 = vit._fp8(a)
    q1, s1 = vit._fp8(a, pm)
    assert torch.equal(q0, q1) and torch.equal(s0, s1)
    L, N, heads = 197, 6, 12
    E = 64 * heads
    qkv = torch.randn(L * N, 3 * E, device=dev, generator=g).bfloat16()
    out = torch.empty(L * N, E, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(L * N * heads, device=dev)
    pm = vit._pmax(dev)
    _hip.call("artsbir_mha_fwd_lse_pmax", _hip.DT_BF16, qkv.data_ptr(), L, N, heads, None, out.data_ptr(),
              lse.data_ptr(), pm.data_ptr(), st)
    q0, s0 = vit._fp8(out)
    q1, s1 = vit._fp8(out, pm)
    assert torch.equal(q0, q1) and torch.equal(s0, s1)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(600, 520, 384), (68, 256, 256)])
def test_fp8_gemm_residual_and_second_output(M, N, K, dev):
    """artsbir_gemm_nt_fp8_ex: bf16 residual input, bf16 copy of the result,
    C read but not written (skip_c) — the ViT block's fused residual adds"""
    import _hip
    import vit
    g = torch.Generator(device=dev).manual_seed(21)
    a = torch.randn(M, K, device=dev, generator=g)
    b = torch.randn(N, K, device=dev, generator=g) * 0.05
    bias = torch.randn(N, device=dev, generator=g)
    qa, sa = vit._fp8(a)
    qb, sb = vit._fp8(b)
    da = qa.view(torch.float8_e4m3fn).double().cpu() * sa.double().cpu()
    db = qb.view(torch.float8_e4m3fn).double().cpu() * sb.double().cpu()
    ref = da @ db.T + bias.double().cpu()
    res = torch.randn(M, N, device=dev, generator=g).bfloat16()
    c = torch.empty(M, N, device=dev)
    out2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    _hip.call("artsbir_gemm_nt_fp8_ex", M, N, K, qa.data_ptr(), qb.data_ptr(), sa.data_ptr(), sb.data_ptr(),
              bias.data_ptr(), c.data_ptr(), _hip.DT_F32, 0, res.data_ptr(), out2.data_ptr(), 0, _hip.stream())
    want = ref + res.double().cpu()
    scale = want.abs().max().item()
    assert (c.double().cpu() - want).abs().max().item() / scale < 5e-5
    assert torch.equal(out2.cpu(), c.cpu().bfloat16())
    # accumulate onto C, skip writing it, only the bf16 copy
    c0 = c.clone()
    out3 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    _hip.call("artsbir_gemm_nt_fp8_ex", M, N, K, qa.data_ptr(), qb.data_ptr(), sa.data_ptr(), sb.data_ptr(),
              bias.data_ptr(), c.data_ptr(), _hip.DT_F32, 1, None, out3.data_ptr(), 1, _hip.stream())
    assert torch.equal(c, c0)
    want3 = c0.double().cpu() + ref
    assert (out3.double().cpu() - want3).abs().max().item() / want3.abs().max().item() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["auto", "0", "3", "11", "12", "13", "16"])
@pytest.mark.parametrize("M,N,K", [(300, 512, 768), (1000, 3072, 768), (4096, 256, 128)])
def test_gemm_nt_gate_matches_gemm_then_quickgelu_bwd(M, N, K, cfg, dev, monkeypatch):
    """artsbir_gemm_nt_gate = (a @ b^T) * quickgelu'(x) (the c_proj input gradient
    through QuickGELU.backward, models.py:391-393) in bf16, with its column sums
    (the c_fc bias gradient) in the statistics slots; ragged M; per tile candidate
    (16: the 128 x 128 tile with the gate operand read from global memory)"""
    import _hip
    if cfg != "auto":
        monkeypatch.setenv("ARTSBIR_PGEMM_CFG", cfg)
    g = torch.Generator(device=dev).manual_seed(31)
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    b = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    x = (torch.randn(M, N, device=dev, generator=g) * 2).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    slots = torch.zeros(_hip.NSLOT, 2, N, device=dev)
    _hip.call("artsbir_gemm_nt_gate", M, N, K, a.data_ptr(), K, b.data_ptr(), out.data_ptr(), N, x.data_ptr(),
              slots.data_ptr(), _hip.stream())
    import _kernels
    _kernels.require(cfg)
    xd = x.double().cpu()
    sg = torch.sigmoid(1.702 * xd)
    ref = (a.double().cpu() @ b.double().cpu().T) * (sg + 1.702 * xd * sg * (1 - sg))
    err = (out.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err  # bf16 output rounding
    colsum = slots[:, 0].sum(0).double().cpu()
    assert ((colsum - ref.sum(0)).norm() / ref.sum(0).norm()).item() < 1e-4


@pytest.mark.gpu
def test_fp8_quantiser_exhaustive_over_bf16(dev):
    """artsbir_quantize_fp8 on every finite bf16 value below a bound (the bound sets
    the tensor's amax, hence the scale) = torch's e4m3fn cast of x / (amax / 448),
    code for code: the fma-corrected reciprocal division and the branch-free
    rounding of fp8.hip against IEEE division and torch's RNE"""
    import vit
    allb = (torch.arange(65536, dtype=torch.int32).to(torch.int16)).view(torch.bfloat16)
    allb = allb[torch.isfinite(allb)]
    for bound in [3.0e38, 448.0, 1.0, 0.3, 7.5e-3, 1.0e-20, 6.0e4]:
        x = allb[allb.float().abs() <= bound].contiguous()
        q, s = vit._fp8(x.to(dev))
        amax = x.float().abs().max()
        want = (x.float() / (amax / 448.0)).to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(q.cpu(), want), (bound, int((q.cpu() != want).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(600, 520, 384), (68, 256, 256), (1000, 3072, 768)])
def test_fp8_gemm_gelu_matches_gemm_then_quickgelu(M, N, K, dev):
    """artsbir_gemm_nt_fp8_gelu = artsbir_gemm_nt_fp8_ex (bf16 f) followed by
    artsbir_quickgelu_pmax on f, bit for bit: f, quickgelu(f) and the quantiser's
    scale from the folded maxima"""
    import vit
    g = torch.Generator(device=dev).manual_seed(41)
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = torch.randn(N, K, device=dev, generator=g) * 0.05
    bias = torch.randn(N, device=dev, generator=g)
    f_ref = vit._gemm_fp8(a, w, bias, out_dtype=torch.bfloat16)
    g_ref = torch.empty_like(f_ref)
    pm_ref = vit._pmax(dev)
    vit.call("artsbir_quickgelu_pmax", vit._dt(f_ref), f_ref.data_ptr(), f_ref.numel(), g_ref.data_ptr(),
             pm_ref.data_ptr(), vit._st())
    pm = vit._pmax(dev)
    f, gg = vit._gemm_fp8_gelu(a, w, bias, None, pm)
    assert torch.equal(f, f_ref)
    assert torch.equal(gg, g_ref)
    assert pm.max().item() == pm_ref.max().item()
    q1, s1 = vit._fp8(gg, pm)
    q2, s2 = vit._fp8(g_ref)
    assert torch.equal(q1, q2) and torch.equal(s1, s2)


@pytest.mark.gpu
@pytest.mark.parametrize("C", [256, 768, 1024, 520])
@pytest.mark.parametrize("rows", [37, 2500])
@pytest.mark.parametrize("sums", [False, True])
def test_layernorm_bwd_bf16_forms(dev, C, rows, sums):
    """artsbir_layernorm_bwd(_sums) on bf16 rows against float64 autograd of the
    oracle LayerNorm on the same (bf16-rounded) inputs: the 4-column form
    (C % 256 == 0, two rows in flight per wave) and the 8-column form (C = 520).
    dx is stored in bf16 (tolerance 1e-2 relative); dgamma / dbeta and the
    column sums of dres and dx are f32 sums over the rows (1e-4)"""
    import _hip
    g = torch.Generator().manual_seed(C + rows)
    x = torch.randn(rows, C, generator=g).bfloat16()
    gam, bet = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g).bfloat16()
    res = torch.randn(rows, C, generator=g).bfloat16()
    xr = x.double().requires_grad_(True)
    gr, br = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    (oenc.layernorm_fp32(xr, gr, br) * dy.double()).sum().backward()
    want_dx = xr.grad + res.double()
    X, G, Dy, Rs = (t.to(dev) for t in (x, gam, dy, res))
    dx = torch.empty_like(X)
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    st = _hip.stream()
    if sums:
        rsum = torch.zeros(C, device=dev)
        xsum = torch.zeros(C, device=dev)
        _hip.call("artsbir_layernorm_bwd_sums", _hip.DT_BF16, X.data_ptr(), G.data_ptr(), Dy.data_ptr(), rows, C,
                  1e-5, Rs.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), rsum.data_ptr(), xsum.data_ptr(),
                  st)
    else:
        _hip.call("artsbir_layernorm_bwd", _hip.DT_BF16, X.data_ptr(), G.data_ptr(), Dy.data_ptr(), rows, C, 1e-5,
                  Rs.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), st)
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(dx, want_dx) < 1e-2
    assert rel(dg, gr.grad) < 1e-4 and rel(db, br.grad) < 1e-4
    if sums:
        assert rel(rsum, res.double().sum(0)) < 1e-4
        assert rel(xsum, want_dx.sum(0)) < 1e-4  # the f32 values before dx's rounding to bf16
