"""Drop-in encoder classes of /root/reference/models.py on MI355X.

Same constructors, attributes and state_dict keys as the reference:
  Bottleneck(inplanes, planes, stride=1)                                  models.py:191-236
  AttentionPool2d(spacial_dim, embed_dim, num_heads, output_dim=None)     models.py:239-272
  ModifiedResNet(layers, output_dim, heads=32, input_resolution=224, width=64)   models.py:275-360
  ModifiedResNet_with_classification(..., num_classes=125, num_classes2=0)     models.py:363-379
  LayerNorm / QuickGELU / ResidualAttentionBlock                          models.py:382-417
The parameters are ordinary torch Parameters in the reference layout (so
``.pth`` checkpoints of the reference load with ``load_state_dict``); the
forward and backward of the encoder run entirely in libartsbir_hip through
``engine.Engine`` (no torch compute kernels, no CPU fallback).

Additions over the reference: ``compute_dtype`` (torch.float32 = the
reference's fp32 semantics, default; torch.bfloat16 = MFMA bf16 throughput
mode with f32 accumulation/statistics/master weights).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

import _hip
import engine as _engine

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class ClipTransform:
    """PIL -> normalised tensor, the compose of models.py:289-295 without
    torchvision: bicubic resize of the shorter side, centre crop, RGB,
    [0,1] float CHW, CLIP normalize."""

    def __init__(self, resolution=224):
        self.resolution = resolution

    def __call__(self, img):
        from PIL import Image
        r = self.resolution
        w, h = img.size
        if w <= h:
            nw, nh = r, int(r * h / w)
        else:
            nw, nh = int(r * w / h), r
        img = img.resize((nw, nh), Image.BICUBIC)
        left, top = int(round((nw - r) / 2.0)), int(round((nh - r) / 2.0))
        img = img.crop((left, top, left + r, top + r)).convert('RGB')
        a = torch.from_numpy(np.asarray(img, dtype=np.float32).copy() / 255.0).permute(2, 0, 1)
        mean = torch.tensor(CLIP_MEAN)[:, None, None]
        std = torch.tensor(CLIP_STD)[:, None, None]
        return (a - mean) / std

    def __repr__(self):
        return f"ClipTransform(resize={self.resolution}, bicubic, center_crop, RGB, ToTensor, Normalize(CLIP))"


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        out = planes * self.expansion
        # all convs have stride 1; an AvgPool after conv2 does the striding
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu2 = nn.ReLU(inplace=True)
        self.avgpool = nn.AvgPool2d(stride) if stride > 1 else nn.Identity()
        self.conv3 = nn.Conv2d(planes, out, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out)
        self.relu3 = nn.ReLU(inplace=True)
        self.downsample = None
        self.stride = stride
        if stride > 1 or inplanes != out:
            self.downsample = nn.Sequential(OrderedDict([
                ("-1", nn.AvgPool2d(stride)),
                ("0", nn.Conv2d(inplanes, out, 1, stride=1, bias=False)),
                ("1", nn.BatchNorm2d(out))]))

    def forward(self, x):
        # inside ModifiedResNet the encoder runs every block itself; called on
        # its own the block runs on the same kernels (engine.ModuleEngine)
        return _module_call(self, x)


class AttentionPool2d(nn.Module):
    def __init__(self, spacial_dim: int, embed_dim: int, num_heads: int, output_dim: int = None):
        super().__init__()
        self.positional_embedding = nn.Parameter(torch.randn(spacial_dim ** 2 + 1, embed_dim) / embed_dim ** 0.5)
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.c_proj = nn.Linear(embed_dim, output_dim or embed_dim)
        self.num_heads = num_heads

    def forward(self, x):
        return _module_call(self, x)


class _ModuleFunction(torch.autograd.Function):
    """one autograd node per standalone Bottleneck / AttentionPool2d call"""

    @staticmethod
    def forward(ctx, x, mod, *params):
        eng = _module_engine(mod)
        out, state = eng.module_forward(x, mod.training)
        ctx.state, ctx.mod, ctx.dtype, ctx.nparams = state, mod, eng.dtype, len(params)
        return out

    @staticmethod
    def backward(ctx, dout):
        eng = _module_engine(ctx.mod)
        eng.dtype = ctx.dtype
        dx = eng.module_backward(ctx.state, dout)
        ctx.state = None
        return (dx, None) + (None,) * ctx.nparams


def _module_engine(mod):
    eng = mod.__dict__.get("_hip_engine")
    if eng is None:
        eng = _engine.ModuleEngine(mod)
        object.__setattr__(mod, "_hip_engine", eng)
    eng.dtype = getattr(mod, "compute_dtype", torch.float32)
    return eng


def _module_call(mod, x):
    params = tuple(mod.parameters())
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        return _ModuleFunction.apply(x, mod, *params)
    out, _ = _module_engine(mod).module_forward(x, mod.training)
    return out


class _EncoderFunction(torch.autograd.Function):
    """One autograd node per encoder call (the reference records ~300 eager
    ops); backward replays the whole encoder backward in libartsbir_hip."""

    @staticmethod
    def forward(ctx, x, model, *params):
        eng = model._hip_engine
        eng.dtype = model.compute_dtype
        out, state = eng.forward(x, model.training, save=True)
        ctx.state, ctx.model, ctx.dtype, ctx.nparams = state, model, model.compute_dtype, len(params)
        return out

    @staticmethod
    def backward(ctx, dout):
        # parameter gradients are accumulated in place into param.grad (views of
        # the engine's flat gradient buffer) by the HIP kernels themselves
        eng = ctx.model._hip_engine
        eng.dtype = ctx.dtype
        eng.backward(ctx.state, dout)
        ctx.state = None
        return (None, None) + (None,) * ctx.nparams


class _EncoderBranchesFunction(torch.autograd.Function):
    """G forward calls of the reference (train.py:28-30) as one autograd node:
    one batched launch per GEMM, BatchNorm statistics per branch."""

    @staticmethod
    def forward(ctx, model, nb, *args):
        xs, params = args[:nb], args[nb:]
        eng = model._hip_engine
        eng.dtype = model.compute_dtype
        out, state = eng.forward(list(xs), model.training, save=True)
        ctx.state, ctx.model, ctx.dtype, ctx.nb, ctx.nparams = state, model, model.compute_dtype, nb, len(params)
        return tuple(out.chunk(nb))

    @staticmethod
    def backward(ctx, *douts):
        ref = next(d for d in douts if d is not None)
        dout = torch.cat([d if d is not None else torch.zeros_like(ref) for d in douts])
        eng = ctx.model._hip_engine
        eng.dtype = ctx.dtype
        eng.backward(ctx.state, dout)
        ctx.state = None
        return (None, None) + (None,) * (ctx.nb + ctx.nparams)


class ModifiedResNet(nn.Module):
    """CLIP ModifiedResNet: 3-conv stem with avgpool, anti-aliased strided
    Bottlenecks, attention-pool head (models.py:275-360)."""

    def __init__(self, layers, output_dim, heads=32, input_resolution=224, width=64):
        super().__init__()
        self.output_dim = output_dim
        self.input_resolution = input_resolution
        self.transform = ClipTransform(input_resolution)
        self.trained_layers = []
        self.compute_dtype = torch.float32

        self.conv1 = nn.Conv2d(3, width // 2, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(width // 2)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(width // 2, width // 2, kernel_size=3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width // 2)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(width // 2, width, kernel_size=3, padding=1, bias=False)
        self.bn3 = nn.BatchNorm2d(width)
        self.relu3 = nn.ReLU(inplace=True)
        self.avgpool = nn.AvgPool2d(2)

        self._inplanes = width
        self.layer1 = self._make_layer(width, layers[0])
        self.layer2 = self._make_layer(width * 2, layers[1], stride=2)
        self.layer3 = self._make_layer(width * 4, layers[2], stride=2)
        self.layer4 = self._make_layer(width * 8, layers[3], stride=2)

        embed_dim = width * 32
        self.attnpool = AttentionPool2d(input_resolution // 32, embed_dim, heads, output_dim)
        object.__setattr__(self, "_hip_engine", _engine.Engine(self))

    def _make_layer(self, planes, blocks, stride=1):
        mods = [Bottleneck(self._inplanes, planes, stride)]
        self._inplanes = planes * Bottleneck.expansion
        mods += [Bottleneck(self._inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def freeze_layers(self):
        self.trained_layers.append('all')

    # ---- engine helpers
    def blocks(self):
        return [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]

    def total_bn_channels(self):
        return sum(m.num_features for m in self.modules() if isinstance(m, nn.BatchNorm2d))

    def grad_order(self):
        """parameter order of the gradient buffer: k/v projections adjacent."""
        ap = self.attnpool
        first = [ap.k_proj.weight, ap.v_proj.weight, ap.k_proj.bias, ap.v_proj.bias]
        ids = {id(p) for p in first}
        return first + [p for p in self.parameters() if id(p) not in ids]

    def encode(self, x):
        params = tuple(self.parameters())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _EncoderFunction.apply(x, self, *params)
        eng = self._hip_engine
        eng.dtype = self.compute_dtype
        return eng.forward(x, self.training, save=False)[0]

    def forward(self, x):
        return self.encode(x)

    def encode_branches(self, xs):
        """[model(x) for x in xs] with the same arithmetic (per-call BatchNorm
        batch statistics, running statistics updated once per call in order)
        but every convolution launched once over all the calls' images."""
        xs = list(xs)
        if len(xs) == 1:
            return [self.encode(xs[0])]
        params = tuple(self.parameters())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return list(_EncoderBranchesFunction.apply(self, len(xs), *xs, *params))
        eng = self._hip_engine
        eng.dtype = self.compute_dtype
        return list(eng.forward(xs, self.training, save=False)[0].chunk(len(xs)))

    def forward_branches(self, xs):
        """the triplet's sketch / positive / negative forwards (train.py:28-30)"""
        return self.encode_branches(xs)


class ModifiedResNet_with_classification(ModifiedResNet):
    def __init__(self, layers, output_dim, heads=32, input_resolution=224, width=64, num_classes=125, num_classes2=0):
        super().__init__(layers, output_dim, heads, input_resolution, width)
        self.num_classes = num_classes
        self.num_classes2 = num_classes2
        self.classifier = nn.Linear(output_dim, num_classes)
        if num_classes2 > 0:
            self.classifier2 = nn.Linear(output_dim, num_classes2)

    def grad_order(self):
        heads = {id(p) for p in self._head_params()}
        return [p for p in super().grad_order() if id(p) not in heads] + list(self._head_params())

    def _head_params(self):
        ps = list(self.classifier.parameters())
        if self.num_classes2 > 0:
            ps += list(self.classifier2.parameters())
        return ps

    def _heads(self, feature):
        import heads as _heads
        classes = _heads.linear(feature, self.classifier.weight, self.classifier.bias)
        if self.num_classes2 == 0:
            return feature, classes
        return feature, classes, _heads.linear(feature, self.classifier2.weight, self.classifier2.bias)

    def forward(self, x):
        return self._heads(super().forward(x))

    def forward_branches(self, xs):
        return [self._heads(f) for f in self.encode_branches(xs)]


# transformer pieces (models.py:382-417) and the ViT-B/16 encoder of C5: vit.py
from vit import LayerNorm, QuickGELU, ResidualAttentionBlock, Transformer, VisionTransformer  # noqa: E402,F401
