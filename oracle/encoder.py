"""CPU fp32 restatement of the CLIP-style ModifiedResNet encoder (TEST ORACLE).

Follows /root/reference/models.py:
  Bottleneck            models.py:191-236
  AttentionPool2d       models.py:239-272  (F.multi_head_attention_forward, q = token 0)
  ModifiedResNet        models.py:275-360  (3-conv stem, avgpool anti-aliasing, attnpool head)
  ..._with_classification models.py:363-379
  LayerNorm / QuickGELU / ResidualAttentionBlock models.py:382-417 (block only;
                        no reference model builds it)
State-dict keys are identical to the reference so checkpoints interchange.
No torchvision: the PIL ``transform`` of models.py:289-295 is not part of the
compute path (synthetic tensors are fed directly).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

EXPANSION = 4

# Test hook (parity tests only): when set, every ReLU of the encoder calls
# RELU(x) instead of F.relu(x), in forward order.  tests/test_c2_gpu.py uses it
# for a MASK-CONDITIONED oracle: x * (the HIP forward's ReLU decision), so the
# float64 gradient is evaluated on the same piecewise-linear branch as the HIP
# one and a comparison measures arithmetic, not ReLU flips at |x| ~ 1e-7.
RELU = None


def _relu(x):
    return F.relu(x) if RELU is None else RELU(x)


def _conv(cin, cout, k, stride=1):
    return nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False)


class Bottleneck(nn.Module):
    """models.py:191-236 — 1x1 -> 3x3 -> [avgpool s] -> 1x1(x4), residual, ReLU."""
    expansion = EXPANSION

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        wide = planes * EXPANSION
        self.conv1, self.bn1, self.relu1 = _conv(inplanes, planes, 1), nn.BatchNorm2d(planes), nn.ReLU()
        self.conv2, self.bn2, self.relu2 = _conv(planes, planes, 3), nn.BatchNorm2d(planes), nn.ReLU()
        self.avgpool = nn.AvgPool2d(stride) if stride > 1 else nn.Identity()
        self.conv3, self.bn3, self.relu3 = _conv(planes, wide, 1), nn.BatchNorm2d(wide), nn.ReLU()
        self.stride = stride
        self.downsample = None
        if stride > 1 or inplanes != wide:
            # keys "-1" (pool), "0" (conv), "1" (bn) as in models.py:216-220
            self.downsample = nn.Sequential(OrderedDict(
                [("-1", nn.AvgPool2d(stride)), ("0", _conv(inplanes, wide, 1)), ("1", nn.BatchNorm2d(wide))]))

    def forward(self, x):
        h = _relu(self.bn1(self.conv1(x)))
        h = self.avgpool(_relu(self.bn2(self.conv2(h))))
        h = self.bn3(self.conv3(h))
        skip = x if self.downsample is None else self.downsample(x)
        return _relu(h + skip)


class AttentionPool2d(nn.Module):
    """models.py:239-272 — mean token + positional embedding, 1-query MHA, c_proj."""

    def __init__(self, spacial_dim, embed_dim, num_heads, output_dim=None):
        super().__init__()
        self.positional_embedding = nn.Parameter(torch.randn(spacial_dim ** 2 + 1, embed_dim) / embed_dim ** 0.5)
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.c_proj = nn.Linear(embed_dim, output_dim or embed_dim)
        self.num_heads = num_heads

    def forward(self, x):
        b, c, h, w = x.shape
        seq = x.reshape(b, c, h * w).permute(2, 0, 1)                # (HW, B, C)
        seq = torch.cat([seq.mean(0, keepdim=True), seq], 0)          # (HW+1, B, C)
        seq = seq + self.positional_embedding[:, None, :].to(seq.dtype)
        out, _ = F.multi_head_attention_forward(
            query=seq[:1], key=seq, value=seq, embed_dim_to_check=c, num_heads=self.num_heads,
            q_proj_weight=self.q_proj.weight, k_proj_weight=self.k_proj.weight,
            v_proj_weight=self.v_proj.weight, in_proj_weight=None,
            in_proj_bias=torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias]),
            bias_k=None, bias_v=None, add_zero_attn=False, dropout_p=0.0,
            out_proj_weight=self.c_proj.weight, out_proj_bias=self.c_proj.bias,
            use_separate_proj_weight=True, training=self.training, need_weights=False)
        return out[0]


class ModifiedResNet(nn.Module):
    """models.py:275-360.  Signature (layers, output_dim, heads=32, input_resolution=224, width=64)."""

    def __init__(self, layers, output_dim, heads=32, input_resolution=224, width=64):
        super().__init__()
        self.output_dim = output_dim
        self.input_resolution = input_resolution
        self.trained_layers = []
        half = width // 2
        self.conv1 = nn.Conv2d(3, half, 3, stride=2, padding=1, bias=False)
        self.bn1, self.relu1 = nn.BatchNorm2d(half), nn.ReLU()
        self.conv2, self.bn2, self.relu2 = _conv(half, half, 3), nn.BatchNorm2d(half), nn.ReLU()
        self.conv3, self.bn3, self.relu3 = _conv(half, width, 3), nn.BatchNorm2d(width), nn.ReLU()
        self.avgpool = nn.AvgPool2d(2)
        inplanes = width
        for i, (mult, nblk) in enumerate(zip((1, 2, 4, 8), layers)):
            blocks = []
            for j in range(nblk):
                blocks.append(Bottleneck(inplanes, width * mult, (1 if i == 0 or j > 0 else 2)))
                inplanes = width * mult * EXPANSION
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.attnpool = AttentionPool2d(input_resolution // 32, width * 32, heads, output_dim)

    def freeze_layers(self):  # models.py:341-342 — bookkeeping only
        self.trained_layers.append('all')

    def forward(self, x):
        x = x.type(self.conv1.weight.dtype)
        for conv, bn in ((self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)):
            x = _relu(bn(conv(x)))
        x = self.avgpool(x)
        for name in ("layer1", "layer2", "layer3", "layer4"):
            x = getattr(self, name)(x)
        return self.attnpool(x)


class ModifiedResNet_with_classification(ModifiedResNet):
    """models.py:363-379 — returns (feature, logits[, logits2])."""

    def __init__(self, layers, output_dim, heads=32, input_resolution=224, width=64, num_classes=125,
                 num_classes2=0):
        super().__init__(layers, output_dim, heads, input_resolution, width)
        self.num_classes, self.num_classes2 = num_classes, num_classes2
        self.classifier = nn.Linear(output_dim, num_classes)
        if num_classes2 > 0:
            self.classifier2 = nn.Linear(output_dim, num_classes2)

    def forward(self, x):
        f = super().forward(x)
        if self.num_classes2 == 0:
            return f, self.classifier(f)
        return f, self.classifier(f), self.classifier2(f)


# ---------------------------------------------------------------------------
# deterministic, portable initialisation (numpy PCG64 -> fp32), used for the
# golden fixtures and for every parity test: the same seed gives the same
# weights on any machine and in the HIP path.
# ---------------------------------------------------------------------------
def layernorm_fp32(x, weight, bias, eps=1e-5):
    """models.py:382-388: LayerNorm evaluated in fp32, result cast back to x's dtype"""
    xf = x.float()
    mu = xf.mean(-1, keepdim=True)
    var = ((xf - mu) ** 2).mean(-1, keepdim=True)
    return ((xf - mu) / torch.sqrt(var + eps) * weight + bias).to(x.dtype)


def quick_gelu(x):
    """models.py:391-393"""
    return x * torch.sigmoid(1.702 * x)


def _linear(a, w, b):
    return a @ w.t() + b


def residual_attention_block(x, sd, n_head, attn_mask=None, eps=1e-5, linear=None):
    """models.py:396-417 on a state dict with the reference keys (attn.in_proj_*,
    attn.out_proj.*, ln_1.*, mlp.c_fc.*, mlp.c_proj.*, ln_2.*): x [L, N, E],
    seq-first; self-attention of nn.MultiheadAttention written out (q scaled by
    1/sqrt(head_dim), additive float mask, softmax over keys).  ``linear(a, w, b)``
    computes the four projections (default a @ w.T + b; the C5 tests pass an
    e4m3-quantising one to price what fp8 operands cost)."""
    linear = linear or _linear
    L, N, E = x.shape
    hd = E // n_head
    h = layernorm_fp32(x, sd["ln_1.weight"], sd["ln_1.bias"], eps)
    qkv = linear(h, sd["attn.in_proj_weight"], sd["attn.in_proj_bias"])
    q, k, v = qkv.split(E, dim=-1)

    def heads(t):  # [L, N, E] -> [N, heads, L, hd]
        return t.reshape(L, N, n_head, hd).permute(1, 2, 0, 3)
    s = (heads(q) / hd ** 0.5) @ heads(k).transpose(-1, -2)
    if attn_mask is not None:
        s = s + attn_mask
    o = (torch.softmax(s, dim=-1) @ heads(v)).permute(2, 0, 1, 3).reshape(L, N, E)
    x = x + linear(o, sd["attn.out_proj.weight"], sd["attn.out_proj.bias"])
    h = layernorm_fp32(x, sd["ln_2.weight"], sd["ln_2.bias"], eps)
    f = quick_gelu(linear(h, sd["mlp.c_fc.weight"], sd["mlp.c_fc.bias"]))
    return x + linear(f, sd["mlp.c_proj.weight"], sd["mlp.c_proj.bias"])


def init_params(model: nn.Module, seed: int = 1234) -> None:
    rng = np.random.Generator(np.random.PCG64(seed))
    with torch.no_grad():
        for name, p in model.named_parameters():
            shape = tuple(p.shape)
            leaf = name.rsplit(".", 1)[-1]
            if name.endswith("positional_embedding"):
                v = rng.standard_normal(shape) / np.sqrt(shape[1])
            elif leaf == "weight" and len(shape) == 1:      # batch-norm gamma
                v = 1.0 + 0.1 * rng.standard_normal(shape)
            elif leaf == "bias":
                v = 0.05 * rng.standard_normal(shape)
            else:                                           # conv / linear weight
                fan_in = int(np.prod(shape[1:]))
                v = rng.standard_normal(shape) / np.sqrt(fan_in)
            p.copy_(torch.from_numpy(v.astype(np.float32)))


def synthetic_triplet(batch: int, res: int, seed: int = 0):
    """SURVEY §8d synthetic inputs: sketch = 90% white / 10% black strokes, photos
    uniform[0,1); both through the CLIP normalize of models.py:294."""
    mean = np.array((0.48145466, 0.4578275, 0.40821073), np.float32)[None, :, None, None]
    std = np.array((0.26862954, 0.26130258, 0.27577711), np.float32)[None, :, None, None]
    out = []
    for i, kind in enumerate(("sketch", "pos", "neg")):
        rng = np.random.Generator(np.random.PCG64(seed * 3 + i))
        if kind == "sketch":
            img = (rng.random((batch, 1, res, res)) >= 0.1).astype(np.float32).repeat(3, axis=1)
        else:
            img = rng.random((batch, 3, res, res), dtype=np.float32)
        out.append(torch.from_numpy(((img - mean) / std).astype(np.float32)))
    return tuple(out)


def vision_transformer(x, sd, patch, n_head, eps=1e-5, linear=None):
    """CLIP's VisionTransformer.forward (the C5 encoder; the reference ships only
    its blocks, models.py:382-417) on a state dict with CLIP's keys: conv1
    patch embedding, class token, positional embedding, ln_pre, resblocks,
    ln_post of the class token, proj.  x [B, 3, R, R] -> [B, output_dim]."""
    B = x.shape[0]
    t = F.conv2d(x, sd["conv1.weight"], stride=patch)                  # [B, E, G, G]
    t = t.reshape(B, t.shape[1], -1).permute(0, 2, 1)                  # [B, P, E]
    cls = sd["class_embedding"].to(t.dtype) + torch.zeros(B, 1, t.shape[-1], dtype=t.dtype)
    t = torch.cat([cls, t], dim=1) + sd["positional_embedding"].to(t.dtype)
    t = layernorm_fp32(t, sd["ln_pre.weight"], sd["ln_pre.bias"], eps)
    t = t.permute(1, 0, 2)                                             # [L, B, E]
    i = 0
    while f"transformer.resblocks.{i}.ln_1.weight" in sd:
        pre = f"transformer.resblocks.{i}."
        t = residual_attention_block(t, {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}, n_head,
                                     eps=eps, linear=linear)
        i += 1
    t = t.permute(1, 0, 2)
    c = layernorm_fp32(t[:, 0, :], sd["ln_post.weight"], sd["ln_post.bias"], eps)
    return c @ sd["proj"]
