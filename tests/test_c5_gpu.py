"""Configuration C5 (BASELINE.json configs[4]): the full-size
ViT-B/16 encoder — VisionTransformer(224, patch 16, width 768, 12 blocks, 12
heads, 768-d) built from the reference's ResidualAttentionBlock
(/root/reference/models.py:382-417) — forward and every parameter gradient on
libartsbir_hip, against the float64 oracle (oracle/encoder.vision_transformer)
on 4 images.

Bars are set by what the arithmetic itself costs, measured on the same weights
and inputs, never by a blanket tolerance:
  f32   vs PyTorch's own fp32 run of the oracle (CPU);
  bf16  vs PyTorch's bf16 path (CPU autocast of the oracle);
  fp8   vs the bf16 path's error PLUS that of an e4m3-emulated oracle: float64
        with the four block projections' operands quantised per tensor
        (amax / 448, round to nearest even), straight-through in the backward —
        the fp8 mode quantises exactly those GEMMs' operands in the forward and
        runs its backward in bf16.
Per parameter: relative L2 error of its gradient, with the norm floored at 1e-3
of the largest parameter-gradient norm (a parameter whose gradient is ~0 is not
judged on its relative noise).  The objective is a fixed random projection of
the 768-d outputs, so no hinge can zero a gradient."""
import pytest
import torch

from oracle import encoder as oenc

pytestmark = pytest.mark.gpu

RES, PATCH, WIDTH, LAYERS, HEADS, OUT = 224, 16, 768, 12, 12, 768
NIMG = 4
FLOOR_REL = 1e-3
# mode -> (factor on the reference path's error, absolute floor) for outputs and gradients
BARS = {"f32": (4.0, 1e-4), "bf16": (3.0, 2e-2), "fp8": (2.0, 4e-2)}


def _threads():
    import os
    return max(1, min(16, len(os.sched_getaffinity(0))))


def c5_state_dict(seed=5):
    """CLIP ViT-B/16-style initialisation (GPT-2-style residual-branch scaling)
    with LayerNorm affines perturbed away from (1, 0)"""
    g = torch.Generator().manual_seed(seed)
    E, L = WIDTH, LAYERS
    sd = {"conv1.weight": torch.randn(E, 3, PATCH, PATCH, generator=g) * (3 * PATCH * PATCH) ** -0.5,
          "class_embedding": E ** -0.5 * torch.randn(E, generator=g),
          "positional_embedding": E ** -0.5 * torch.randn((RES // PATCH) ** 2 + 1, E, generator=g)}

    def ln(name):
        sd[name + ".weight"] = 1 + 0.1 * torch.randn(E, generator=g)
        sd[name + ".bias"] = 0.1 * torch.randn(E, generator=g)
    ln("ln_pre")
    for i in range(L):
        p = f"transformer.resblocks.{i}."
        sd[p + "attn.in_proj_weight"] = torch.randn(3 * E, E, generator=g) * E ** -0.5
        sd[p + "attn.in_proj_bias"] = 0.02 * torch.randn(3 * E, generator=g)
        sd[p + "attn.out_proj.weight"] = torch.randn(E, E, generator=g) * (E * 2 * L) ** -0.5
        sd[p + "attn.out_proj.bias"] = 0.02 * torch.randn(E, generator=g)
        ln(p + "ln_1")
        sd[p + "mlp.c_fc.weight"] = torch.randn(4 * E, E, generator=g) * E ** -0.5
        sd[p + "mlp.c_fc.bias"] = 0.02 * torch.randn(4 * E, generator=g)
        sd[p + "mlp.c_proj.weight"] = torch.randn(E, 4 * E, generator=g) * (4 * E * 2 * L) ** -0.5
        sd[p + "mlp.c_proj.bias"] = 0.02 * torch.randn(E, generator=g)
        ln(p + "ln_2")
    ln("ln_post")
    sd["proj"] = E ** -0.5 * torch.randn(E, OUT, generator=g)
    return sd


def _q8(t):
    """per-tensor e4m3 quantise-dequantise (scale amax / 448, RNE), straight-through"""
    s = t.detach().abs().max() / 448.0
    q = (t.detach() / s).to(torch.float8_e4m3fn).to(t.dtype) * s
    return t + (q - t.detach())


def fp8_linear(a, w, b):
    return _q8(a) @ _q8(w).t() + b


def _run(sd, x, wout, dt, autocast=False, linear=None):
    sdr = {k: v.to(dt).clone().requires_grad_(True) for k, v in sd.items()}
    if autocast:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            y = oenc.vision_transformer(x.to(dt), sdr, PATCH, HEADS, linear=linear)
    else:
        y = oenc.vision_transformer(x.to(dt), sdr, PATCH, HEADS, linear=linear)
    (y.double() * wout).sum().backward()
    return y.detach().double(), {k: v.grad.double() for k, v in sdr.items()}


@pytest.fixture(scope="module")
def c5_oracle():
    torch.set_num_threads(_threads())
    sd = c5_state_dict()
    s, p, _ = oenc.synthetic_triplet(NIMG // 2, RES, seed=9)  # sketches and photos
    x = torch.cat([s, p])
    wout = torch.randn(NIMG, OUT, generator=torch.Generator().manual_seed(10), dtype=torch.float64)
    out = {"sd": sd, "x": x, "w": wout}
    out["64"] = _run(sd, x, wout, torch.float64)
    out["32"] = _run(sd, x, wout, torch.float32)
    out["ac"] = _run(sd, x, wout, torch.float32, autocast=True)
    out["fp8emu"] = _run(sd, x, wout, torch.float64, linear=fp8_linear)
    return out


def _rel(a, b, floor=0.0):
    return float((a - b).norm() / max(b.norm().item(), floor, 1e-30))


def _errors(y, grads, ref):
    """output rel-L2 and per-parameter floored rel-L2 against the float64 oracle"""
    y64, g64 = ref["64"]
    floor = FLOOR_REL * max(g.norm().item() for g in g64.values())
    return _rel(y, y64), {k: _rel(grads[k], g64[k], floor) for k in g64}


@pytest.mark.parametrize("mode", ["f32", "bf16", "fp8"])
def test_c5_vit_b16_matches_oracle(mode, c5_oracle, dev):
    import models
    ref = c5_oracle
    m = models.VisionTransformer(RES, PATCH, WIDTH, LAYERS, HEADS, OUT)
    m.load_state_dict(ref["sd"], strict=True)
    m = m.to(dev)
    m.compute_dtype = {"f32": torch.float32, "bf16": torch.bfloat16, "fp8": "fp8"}[mode]
    m.train()
    y = m(ref["x"].to(dev))
    assert y.dtype == torch.float32 and y.shape == (NIMG, OUT)
    (y * ref["w"].float().to(dev)).sum().backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    e_y, e_g = _errors(y.detach().double().cpu(), grads, ref)
    # the reference path's own error on the same weights and inputs
    if mode == "f32":
        r_y, r_g = _errors(*ref["32"], ref)
    else:
        r_y, r_g = _errors(*ref["ac"], ref)
        if mode == "fp8":
            q_y, q_g = _errors(*ref["fp8emu"], ref)
            r_y, r_g = r_y + q_y, {k: r_g[k] + q_g[k] for k in r_g}
    factor, floor = BARS[mode]
    worst = max((e_g[k] / max(floor, factor * r_g[k]), k) for k in e_g)
    print(f"\nC5 {mode}: output rel-L2 {e_y:.3e} (reference path {r_y:.3e}); worst gradient "
          f"{worst[1]}: {e_g[worst[1]]:.3e} (reference path {r_g[worst[1]]:.3e}, bar "
          f"{max(floor, factor * r_g[worst[1]]):.3e}); median gradient error "
          f"{sorted(e_g.values())[len(e_g) // 2]:.3e}")
    assert e_y < max(floor, factor * r_y), (e_y, r_y)
    bad = [(k, e_g[k], r_g[k]) for k in e_g if e_g[k] > max(floor, factor * r_g[k])]
    assert not bad, bad[:8]


def test_c5_step_loss_bf16_fp8_vs_f32(c5_oracle, dev):
    """the C5 training step's loss (3 branches as one batch, TripletMarginLoss(0.2),
    train.py:27-37) in bf16 and fp8 against the f32 mode of the same library on
    the same batch and weights (what bench.py's C5 leg checks at step 0)"""
    import losses
    import models
    ref = c5_oracle
    m = models.VisionTransformer(RES, PATCH, WIDTH, LAYERS, HEADS, OUT)
    m.load_state_dict(ref["sd"], strict=True)
    m = m.to(dev).train()
    x = ref["x"].to(dev)
    xs = [x[:2], x[2:], x.flip(0)[:2]]
    loss_fn = losses.TripletMarginLoss(margin=0.2)
    out, scale = {}, None
    with torch.no_grad():
        for mode in ("f32", "bf16", "fp8"):
            m.compute_dtype = {"f32": torch.float32, "bf16": torch.bfloat16, "fp8": "fp8"}[mode]
            a, p, n = m.forward_branches(xs)
            out[mode] = float(loss_fn(a, p, n).item())
            if mode == "f32":  # the hinge's argument is a difference of distances of this size
                scale = float(((a - p).norm(dim=1) + (a - n).norm(dim=1)).mean())
    print(f"\nC5 step-0 loss: {out}, mean d(a,p) + d(a,n) = {scale:.4f}")
    assert abs(out["bf16"] - out["f32"]) < 1e-2 * scale, (out, scale)
    assert abs(out["fp8"] - out["f32"]) < 4e-2 * scale, (out, scale)
