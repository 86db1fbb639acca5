"""bn1 folded through conv1 with its own input (csrc/fold.hip, the y-side fold;
artsbir_conv1x1_dgrad_fold_y).  The reference differentiates conv1 -> bn1
(models.py:198-199) by autograd: dy1 = c1 (g - c2 - xhat c3), dx = dy1 W (+ the
residual branch's gradient, models.py:234), dW = dy1^T x.  Here dy1 is never
formed: dx = [g | y] w_s^T + bias_s with per-segment weights diag(c1) W | diag(b') W,
and dW from g^T x, y^T x and the column sums of x.  Checked against that chain in
float64 on the CPU, with the block-input BN reduction of the previous block fused
into the epilogue (kind 3 bits / kind 0 mask, one or two targets) and every
two-operand kernel forced in turn (the name of the kernel that ran is asserted)."""
import copy
import os

import pytest
import torch

import _hip

pytestmark = pytest.mark.gpu

# forced candidate -> the kernel it must launch for (plain, fused kind 0/3)
FOLD_Y_KERNELS = {
    "16": ("pgemm_kernel<128,128,k32,glb,fold>", "pgemm_kernel<128,128,k32,glb,bnb,fold>"),
    "18": (None, "pgemm_kernel<256,128,k32,glb,bnb,fold>"),
    "22": ("pp256_kernel<fold>", "pp256_kernel<bnb,fold>"),
    "2": ("pgemm_kernel<256,64,fold>", None),
    "19": ("pgemm_kernel<256,128,k32,glb,fold>", None),
}

CASES = [
    # images per segment, segments, H, W, Co (planes: g, y channels), Ci (inplanes: dx channels), res_mode
    (2, 3, 16, 16, 64, 256, 1),     # layer-1 conv1 family (K = 128)
    (4, 3, 8, 8, 128, 512, 1),      # 256 px / segment: layer-2 conv1
    (2, 3, 16, 16, 128, 256, 2),    # the first block of a strided layer: the downsample's gradient unpooled
    (4, 3, 7, 7, 512, 2048, 1),     # 196 px / segment: tiles straddle segments
    (2, 1, 14, 14, 256, 1024, 1),   # one segment
]


@pytest.fixture
def cfg_env():
    old = os.environ.get("ARTSBIR_PGEMM_CFG")
    yield
    if old is None:
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)
    else:
        os.environ["ARTSBIR_PGEMM_CFG"] = old


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _problem(case, seed, dtype):
    Bs, G, H, W, Co, Ci, res_mode = case
    g = torch.Generator().manual_seed(seed)
    B = Bs * G
    bf = (lambda t: t.to(dtype).double())
    gr = bf(torch.randn(B, H, W, Co, generator=g))                 # masked gradient at bn1's output
    x = bf(torch.relu(torch.randn(B, H, W, Ci, generator=g)))      # the block input (post-ReLU)
    w = bf(torch.randn(Co, Ci, generator=g) / Ci ** 0.5)           # conv1 weight [Co][Ci]
    y = bf((x.reshape(B, -1, Ci) @ w.T).float()).reshape(B, H, W, Co)  # bn1's input, stored in the compute dtype
    ys = y.reshape(G, -1, Co)
    prm = torch.zeros(G, 4, Co)
    prm[:, 0] = ys.mean(1).float()
    prm[:, 1] = (1.0 / (ys.var(1, unbiased=False) + 1e-5).sqrt()).float()
    coef = torch.stack([torch.rand(G, Co, generator=g) + 0.5, torch.randn(G, Co, generator=g) * 0.1,
                        torch.randn(G, Co, generator=g) * 0.1], 1).float()  # c1, c2, c3
    p = 2 if res_mode == 2 else 1
    res = bf(torch.randn(B, H // p, W // p, Ci, generator=g))
    return gr, x, w, y, prm, coef, res


def _dy(gr, y, prm, coef, G):
    Co = gr.shape[-1]
    c = coef.double()
    mean, istd = prm[:, 0].double()[:, None], prm[:, 1].double()[:, None]
    return c[:, 0][:, None] * (gr.reshape(G, -1, Co) - c[:, 1][:, None]
                               - (y.reshape(G, -1, Co) - mean) * istd * c[:, 2][:, None])


def _reference_dx(gr, y, w, prm, coef, res, res_mode, G):
    B, H, W, _ = gr.shape
    dx = (_dy(gr, y, prm, coef, G) @ w).reshape(B, H, W, -1)
    if res_mode == 1:
        dx = dx + res
    elif res_mode == 2:
        dx = dx + 0.25 * res.repeat_interleave(2, 1).repeat_interleave(2, 2)
    return dx


def _prep_y(w, coef, prm, G, dtype, dev):
    Co, Ci = w.shape
    wt = w.T.contiguous().to(dev, dtype)                          # the data-gradient operand W^T [Ci][Co]
    wout = torch.empty(G, Ci, 2 * Co, dtype=dtype, device=dev)
    bias = torch.empty(G, Ci, dtype=torch.float32, device=dev)
    cd, pd = coef.to(dev), prm.to(dev)
    _hip.call("artsbir_bn_fold_bwd_prep_y", _hip.dtype_code(dtype), Co, Ci, wt.data_ptr(), cd.data_ptr(),
              pd.data_ptr(), 4 * Co, G, wout.data_ptr(), bias.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    return wout, bias, (wt, cd, pd)


def _block_input_desc(kind, nt, B, G, H, W, Ci, dtype, dev, seed=31):
    """the fused reduction of the BN(s) at the block input (the previous block's
    bn3 and downsample BN): kind 3 = the block output's ReLU mask as bits, kind 0
    = the block output itself as the mask"""
    g = torch.Generator().manual_seed(seed)
    ys = [torch.randn(B, H, W, Ci, generator=g).to(dtype).double() for _ in range(nt)]
    prm = [torch.zeros(G, 4, Ci) for _ in range(nt)]
    for p in prm:
        p[:, 0] = torch.randn(G, Ci, generator=g) * 0.1
        p[:, 1] = torch.rand(G, Ci, generator=g) + 0.5
    keep = torch.rand(B, H, W, Ci, generator=g) > 0.4
    yd = [t.to(dev, dtype) for t in ys]
    pd = [p.to(dev) for p in prm]
    slots = [torch.zeros(G, _hip.NSLOT, 2, Ci, device=dev) for _ in range(nt)]
    desc = _hip.BnBwdDesc()
    desc.dtype, desc.kind, desc.pool, desc.ntarget = _hip.dtype_code(dtype), kind, 0, nt
    if kind == 3:
        wts = (2 ** torch.arange(8)).to(torch.int32)
        bits = (keep.reshape(-1, Ci // 8, 8).to(torch.int32) * wts).sum(-1).to(torch.uint8).to(dev)
        mask = bits
    else:
        mask = torch.where(keep, 1.0, 0.0).to(dev, dtype)
    desc.mask = mask.data_ptr()
    for t in range(nt):
        desc.y[t] = yd[t].data_ptr()
        desc.mean[t] = pd[t].data_ptr()
        desc.istd[t] = pd[t][0, 1].data_ptr()
        desc.slots[t] = slots[t].data_ptr()
    desc.B, desc.H, desc.W, desc.C = B, H, W, Ci
    return desc, (ys, prm, keep, slots, yd, pd, mask)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_fold_prep_y_matches_formula(dtype, dev):
    case = (2, 3, 8, 8, 128, 512, 1)
    G = case[1]
    gr, x, w, y, prm, coef, res = _problem(case, 1, dtype)
    wout, bias, _ = _prep_y(w, coef, prm, G, dtype, dev)
    c = coef.double()
    mean, istd = prm[:, 0].double(), prm[:, 1].double()
    bp = -c[:, 0] * c[:, 2] * istd
    k = -c[:, 0] * (c[:, 1] - c[:, 2] * istd * mean)
    tol = 1e-6 if dtype == torch.float32 else 4e-3
    out = wout.double().cpu()
    assert _rel(out[:, :, :128], c[:, 0][:, None, :] * w.T[None]) < tol
    assert _rel(out[:, :, 128:], bp[:, None, :] * w.T[None]) < tol
    assert _rel(bias.double().cpu(), torch.einsum("ci,gc->gi", w, k)) < 1e-5


@pytest.mark.parametrize("fused", ["none", "k3t1", "k3t2", "k0t1", "k0t2"])
@pytest.mark.parametrize("cfg", ["auto", "16", "18", "22", "2", "19"])
@pytest.mark.parametrize("case", CASES)
def test_dgrad_fold_y(case, cfg, fused, dev, cfg_env):
    """dx = dy1 W + residual without dy1, against the reference chain in float64;
    with `fused` the previous block's output-BN reduction in the epilogue (g' = dx *
    mask, Σg', Σg'·x̂_t per target)"""
    dtype = torch.bfloat16
    Bs, G, H, W, Co, Ci, res_mode = case
    B = Bs * G
    gr, x, w, y, prm, coef, res = _problem(case, 7, dtype)
    wout, bias, keep_ = _prep_y(w, coef, prm, G, dtype, dev)
    ref = _reference_dx(gr, y, w, prm, coef, res, res_mode, G)
    if cfg == "auto":
        os.environ.pop("ARTSBIR_PGEMM_CFG", None)
    else:
        os.environ["ARTSBIR_PGEMM_CFG"] = cfg
    gd, yd, rd = gr.to(dev, dtype), y.to(dev, dtype), res.to(dev, dtype)
    dx = torch.full((B, H, W, Ci), float("nan"), dtype=dtype, device=dev)
    d = _hip.conv_desc(dtype, B, H, W, Ci, Co, 1, 1, 1, 0)
    desc, aux = (None, None)
    if fused != "none":
        desc, aux = _block_input_desc(int(fused[1]), int(fused[3]), B, G, H, W, Ci, dtype, dev)
    _hip.call("artsbir_conv1x1_dgrad_fold_y", d, gd.data_ptr(), yd.data_ptr(), wout.data_ptr(), bias.data_ptr(),
              dx.data_ptr(), rd.data_ptr(), res_mode, desc, G, 4 * Ci, _hip.stream())
    torch.cuda.synchronize()
    name = _hip.lib().artsbir_last_kernel().decode()
    if cfg != "auto":
        want = FOLD_Y_KERNELS[cfg][0 if fused == "none" else 1]
        # a forced candidate that does not take this case (segment straddling, kind,
        # target count) leaves it to the fallback: never to a differently named fold kernel
        assert "fold" not in name or name == want, (cfg, name, want)
    else:
        assert name.endswith("fold>"), name  # a two-operand kernel, not the concatenated fallback
    out = dx.double().cpu()
    assert torch.isfinite(out).all()
    if aux is not None:
        ys, prms, keep, slots = aux[:4]
        ref = ref * keep
        rg = ref.reshape(G, -1, Ci)
        for t in range(len(ys)):
            xh = (ys[t].reshape(G, -1, Ci) - prms[t][:, 0].double()[:, None]) * prms[t][:, 1].double()[:, None]
            s = slots[t].double().cpu().sum(1)
            assert _rel(s[:, 0], rg.sum(1)) < 2e-2
            assert _rel(s[:, 1], (rg * xh).sum(1)) < 2e-2
    assert _rel(out, ref) < 1.5e-2, _rel(out, ref)


@pytest.mark.parametrize("cfg,case,fused", [
    ("16", CASES[1], "none"), ("16", CASES[1], "k3t2"), ("16", CASES[2], "k0t1"),
    ("18", CASES[0], "k3t1"), ("18", CASES[2], "k3t1"),
    ("22", CASES[4], "k3t1"), ("22", CASES[1], "k0t2"), ("22", CASES[0], "none"),
    ("2", CASES[0], "none"), ("19", CASES[1], "none")])
def test_dgrad_fold_y_candidate_runs(cfg, case, fused, dev, cfg_env):
    """each two-operand kernel really runs (by name) on a shape it takes"""
    dtype = torch.bfloat16
    Bs, G, H, W, Co, Ci, res_mode = case
    B = Bs * G
    gr, x, w, y, prm, coef, res = _problem(case, 3, dtype)
    wout, bias, keep_ = _prep_y(w, coef, prm, G, dtype, dev)
    ref = _reference_dx(gr, y, w, prm, coef, res, res_mode, G)
    os.environ["ARTSBIR_PGEMM_CFG"] = cfg
    gd, yd, rd = gr.to(dev, dtype), y.to(dev, dtype), res.to(dev, dtype)
    dx = torch.empty(B, H, W, Ci, dtype=dtype, device=dev)
    d = _hip.conv_desc(dtype, B, H, W, Ci, Co, 1, 1, 1, 0)
    desc, aux = (None, None)
    if fused != "none":
        desc, aux = _block_input_desc(int(fused[1]), int(fused[3]), B, G, H, W, Ci, dtype, dev)
        ref = ref * aux[2]
    _hip.call("artsbir_conv1x1_dgrad_fold_y", d, gd.data_ptr(), yd.data_ptr(), wout.data_ptr(), bias.data_ptr(),
              dx.data_ptr(), rd.data_ptr(), res_mode, desc, G, 4 * Ci, _hip.stream())
    torch.cuda.synchronize()
    name = _hip.lib().artsbir_last_kernel().decode()
    assert name == FOLD_Y_KERNELS[cfg][0 if fused == "none" else 1], name
    assert _rel(dx.double().cpu(), ref) < 1.5e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("case", [CASES[0], CASES[2], (2, 3, 7, 7, 64, 128, 1)])
@pytest.mark.parametrize("fused", ["none", "k0t1"])
def test_dgrad_fold_y_fallback_and_f32(case, dtype, fused, dev, cfg_env):
    """f32 (the parity mode) and shapes without a two-operand kernel: the
    concatenated operand and one plain GEMM per segment (residual, per-segment
    mask and BN slots sliced per segment)"""
    os.environ["ARTSBIR_PGEMM_CFG"] = "-2" if dtype == torch.bfloat16 else "0"
    Bs, G, H, W, Co, Ci, res_mode = case
    B = Bs * G
    gr, x, w, y, prm, coef, res = _problem(case, 5, dtype)
    wout, bias, keep_ = _prep_y(w, coef, prm, G, dtype, dev)
    ref = _reference_dx(gr, y, w, prm, coef, res, res_mode, G)
    gd, yd, rd = gr.to(dev, dtype), y.to(dev, dtype), res.to(dev, dtype)
    dx = torch.empty(B, H, W, Ci, dtype=dtype, device=dev)
    d = _hip.conv_desc(dtype, B, H, W, Ci, Co, 1, 1, 1, 0)
    desc, aux = (None, None)
    if fused != "none":
        desc, aux = _block_input_desc(0, 1, B, G, H, W, Ci, dtype, dev)
        ref = ref * aux[2]
    _hip.call("artsbir_conv1x1_dgrad_fold_y", d, gd.data_ptr(), yd.data_ptr(), wout.data_ptr(), bias.data_ptr(),
              dx.data_ptr(), rd.data_ptr(), res_mode, desc, G, 4 * Ci, _hip.stream())
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1.5e-2
    assert _rel(dx.double().cpu(), ref) < tol
    if aux is not None:
        ys, prms, keep, slots = aux[:4]
        rg = ref.reshape(G, -1, Ci)
        xh = (ys[0].reshape(G, -1, Ci) - prms[0][:, 0].double()[:, None]) * prms[0][:, 1].double()[:, None]
        s = slots[0].double().cpu().sum(1)
        assert _rel(s[:, 0], rg.sum(1)) < max(tol, 1e-4) * 2
        assert _rel(s[:, 1], (rg * xh).sum(1)) < max(tol, 1e-4) * 2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("case", [CASES[0], CASES[3]])
def test_wgrad_fold_y(case, dtype, dev):
    """dW = dy1^T x from g^T x and y^T x (one artsbir_gemm_tn2 per segment) and the
    column sums of x per segment (replica rows), artsbir_bn_fold_wgrad_combine_y"""
    Bs, G, H, W, Co, Ci, _ = case
    gr, x, w, y, prm, coef, res = _problem(case, 11, dtype)
    dy = _dy(gr, y, prm, coef, G)
    xs = x.reshape(G, -1, Ci)
    ref = torch.einsum("gpc,gpi->ci", dy, xs)
    Ms = xs.shape[1]
    gd, yd, xd = gr.to(dev, dtype), y.to(dev, dtype), x.to(dev, dtype)
    P = torch.zeros(G, Co, Ci, device=dev)
    Q = torch.zeros(G, Co, Ci, device=dev)
    for s in range(G):
        _hip.call("artsbir_gemm_tn2", _hip.dtype_code(dtype), Ms, Co, Co, Ci, gd[s * Bs:].data_ptr(), Co,
                  yd[s * Bs:].data_ptr(), Co, xd[s * Bs:].data_ptr(), Ci, P[s].data_ptr(), Q[s].data_ptr(),
                  _hip.stream())
    cs = xs.sum(1).float()
    cs3 = torch.stack([cs * 0.25, cs * 0.5, cs * 0.25], 1).contiguous().to(dev)
    init = torch.randn(Co, Ci)
    dw = init.clone().to(dev)
    cd, pd = coef.to(dev), prm.to(dev)
    _hip.call("artsbir_bn_fold_wgrad_combine_y", Co, Ci, G, P.data_ptr(), Q.data_ptr(), cs3.data_ptr(), 3,
              cd.data_ptr(), pd.data_ptr(), 4 * Co, dw.data_ptr(), _hip.stream())
    torch.cuda.synchronize()
    assert _rel(dw.double().cpu() - init.double(), ref) < (1e-5 if dtype == torch.float32 else 1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("rows,C,G,ds", [(6 * 256, 256, 3, True), (3 * 784, 512, 3, False), (2 * 49, 2048, 1, True),
                                         (4 * 100, 1024, 2, False)])
def test_block_out_colsum(rows, C, G, ds, dtype, dev):
    """artsbir_block_out_colsum: the block tail of artsbir_block_out_mask (same
    output, same mask bits) plus the per-segment column sums of the stored output"""
    g = torch.Generator().manual_seed(37)
    y3 = torch.randn(rows, C, generator=g).to(dtype).to(dev)
    yd = torch.randn(rows, C, generator=g).to(dtype).to(dev)
    idn = torch.randn(rows, C, generator=g).to(dtype).to(dev)
    bn3, bnd = torch.zeros(G, 4, C), torch.zeros(G, 4, C)
    for p in (bn3, bnd):
        p[:, 0] = torch.randn(G, C, generator=g) * 0.2
        p[:, 2] = torch.rand(G, C, generator=g) + 0.5
        p[:, 3] = torch.randn(G, C, generator=g) * 0.3
    bn3, bnd = bn3.to(dev), bnd.to(dev)
    out, out2 = torch.empty_like(y3), torch.empty_like(y3)
    bits = torch.empty(rows * C // 8, dtype=torch.uint8, device=dev) if dtype == torch.bfloat16 else None
    bits2 = torch.empty_like(bits) if bits is not None else None
    cs = torch.zeros(G, _hip.NSLOT, C, device=dev)
    dt = _hip.dtype_code(dtype)
    args = (y3.data_ptr(), bn3.data_ptr(), yd.data_ptr() if ds else None, bnd.data_ptr() if ds else None,
            None if ds else idn.data_ptr(), rows, C, G)
    _hip.call("artsbir_block_out_colsum", dt, *args, out.data_ptr(), bits.data_ptr() if bits is not None else None,
              cs.data_ptr(), _hip.stream())
    _hip.call("artsbir_block_out_mask", dt, *args, out2.data_ptr(), bits2.data_ptr() if bits2 is not None else None,
              _hip.stream())
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    if bits is not None:
        assert torch.equal(bits, bits2)
    o = out.double().cpu().reshape(G, -1, C)
    assert _rel(cs.double().cpu().sum(1), o.sum(1)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_engine_fold1_toggle_small_resnet(dtype, dev, cfg_env):
    """the engine glue of the y-side fold end to end: one training step of a small
    ModifiedResNet((2,1,1,1), width 64) on G = 3 BN segments with bn1 folded
    through conv1 (engine.FOLD_BN1) against the same step with dy1 formed by the
    apply pass (the block-output fold on in both).  Deterministic mode, so both
    runs take the same ReLU decisions; covers the block_out column sums, the
    reduce-only pass that writes g1, the side-stream combine, the stride-2 blocks'
    unpool residual and a block without a downsample (layer 1's second block)."""
    import engine
    import models
    os.environ.pop("ARTSBIR_PGEMM_CFG", None)
    torch.manual_seed(22)
    base = models.ModifiedResNet((2, 1, 1, 1), 64, heads=32, input_resolution=64, width=64)
    gen = torch.Generator(device=dev).manual_seed(6)
    xs = [torch.randn(2, 3, 64, 64, device=dev, generator=gen) + 0.3 * i for i in range(3)]
    proj = [torch.randn(2, 64, device=dev, generator=gen) for _ in range(3)]

    def run(fold1):
        m = copy.deepcopy(base)
        m.compute_dtype = dtype
        m = m.to(dev)
        m.train()
        trace = []
        old = engine.set_deterministic(True)
        oldf = engine.FOLD_BN1[0]
        engine.FOLD_BN1[0] = fold1
        try:
            _hip.TRACE = trace
            outs = m.forward_branches(xs)
            loss = sum((o * r).sum() for o, r in zip(outs, proj))
            loss.backward()
            torch.cuda.synchronize()
        finally:
            _hip.TRACE = None
            engine.FOLD_BN1[0] = oldf
            engine.set_deterministic(old)
        grads = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
        return torch.cat(outs).detach(), grads, trace

    e0, g0, t0 = run(False)
    assert not [t for t in t0 if t[0] == "artsbir_conv1x1_dgrad_fold_y"]
    e1, g1, t1 = run(True)
    assert torch.equal(e1, e0)  # the forward (with the block-input column sums) is unchanged
    folds = [t for t in t1 if t[0] == "artsbir_conv1x1_dgrad_fold_y"]
    assert len(folds) == 5, folds                                 # one per Bottleneck
    assert len([t for t in t1 if t[0] == "artsbir_bn_fold_wgrad_combine_y"]) == 5
    assert len([t for t in t1 if t[0] == "artsbir_block_out_colsum"]) == 5
    # the apply passes of bn1 are gone: one bn_bwd_apply fewer per block
    n_apply = lambda t: len([u for u in t if u[0] == "artsbir_bn_bwd_apply"])  # noqa: E731
    assert n_apply(t0) - n_apply(t1) == 5, (n_apply(t0), n_apply(t1))
    floor = 1e-4 * max(g.norm().item() for g in g0.values())
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    for k, g in g0.items():
        err = (g1[k] - g).norm().item() / max(g.norm().item(), floor)
        assert err < tol, (k, err)
