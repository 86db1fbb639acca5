"""Independent float64 numpy restatement of the forward math (TEST ORACLE).

Used only to cross-pin oracle/encoder.py + oracle/steps.py (which run the same
torch.nn ops as the reference): two restatements written from the reference
text in different frameworks must agree before either is trusted.
  conv / BatchNorm2d(train) / ReLU / AvgPool2d   models.py:197-236,310-319
  AttentionPool2d                                models.py:249-272
  TripletMarginLoss                              train.py:169
  Adam (coupled weight decay)                    train.py:158
"""
from __future__ import annotations

import numpy as np


def conv2d(x, w, stride=1, pad=0):
    n, c, h, wd = x.shape
    co, _, r, s = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    ho = (h + 2 * pad - r) // stride + 1
    wo = (wd + 2 * pad - s) // stride + 1
    out = np.zeros((n, co, ho, wo))
    for i in range(r):
        for j in range(s):
            patch = xp[:, :, i:i + stride * ho:stride, j:j + stride * wo:stride]  # n c ho wo
            out += np.einsum("nchw,oc->nohw", patch, w[:, :, i, j])
    return out


def batchnorm_train(x, gamma, beta, eps=1e-5):
    mean = x.mean(axis=(0, 2, 3))
    var = x.var(axis=(0, 2, 3))
    cnt = x.shape[0] * x.shape[2] * x.shape[3]
    y = (x - mean[None, :, None, None]) / np.sqrt(var[None, :, None, None] + eps)
    y = y * gamma[None, :, None, None] + beta[None, :, None, None]
    return y, mean, var * cnt / max(cnt - 1, 1)


def batchnorm_eval(x, gamma, beta, rm, rv, eps=1e-5):
    return (x - rm[None, :, None, None]) / np.sqrt(rv[None, :, None, None] + eps) * gamma[None, :, None, None] \
        + beta[None, :, None, None]


def avgpool2(x, k=2):
    n, c, h, w = x.shape
    return x[:, :, :h // k * k, :w // k * k].reshape(n, c, h // k, k, w // k, k).mean(axis=(3, 5))


def relu(x):
    return np.maximum(x, 0)


def attnpool(x, sd, prefix, heads):
    n, c, h, w = x.shape
    tok = x.reshape(n, c, h * w).transpose(0, 2, 1)             # n t c
    tok = np.concatenate([tok.mean(1, keepdims=True), tok], 1) + sd[prefix + "positional_embedding"][None]
    lin = lambda t, nm: t @ sd[f"{prefix}{nm}.weight"].T + sd[f"{prefix}{nm}.bias"]
    q = lin(tok[:, :1], "q_proj")                                 # n 1 c
    k, v = lin(tok, "k_proj"), lin(tok, "v_proj")                 # n t c
    hd = c // heads
    q = q.reshape(n, 1, heads, hd).transpose(0, 2, 1, 3)
    k = k.reshape(n, -1, heads, hd).transpose(0, 2, 1, 3)
    v = v.reshape(n, -1, heads, hd).transpose(0, 2, 1, 3)
    s = q @ k.transpose(0, 1, 3, 2) / np.sqrt(hd)                 # n h 1 t
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    o = (p @ v).transpose(0, 2, 1, 3).reshape(n, c)
    return lin(o, "c_proj")


def encoder_forward(x, sd, layers, heads, train=True):
    """Full ModifiedResNet forward from a float64 state dict (dict of np arrays).
    Returns (embedding, batch statistics {bn_prefix: (mean, unbiased var)})."""
    stats = {}

    def bn(t, p):
        if train:
            y, m, uv = batchnorm_train(t, sd[p + ".weight"], sd[p + ".bias"])
            stats[p] = (m, uv)
            return y
        return batchnorm_eval(t, sd[p + ".weight"], sd[p + ".bias"], sd[p + ".running_mean"], sd[p + ".running_var"])

    h = x
    for i, st in ((1, 2), (2, 1), (3, 1)):
        h = relu(bn(conv2d(h, sd[f"conv{i}.weight"], st, 1), f"bn{i}"))
    h = avgpool2(h)
    for li, nblk in enumerate(layers):
        for b in range(nblk):
            p = f"layer{li + 1}.{b}."
            stride = 2 if (li > 0 and b == 0) else 1
            o = relu(bn(conv2d(h, sd[p + "conv1.weight"]), p + "bn1"))
            o = relu(bn(conv2d(o, sd[p + "conv2.weight"], 1, 1), p + "bn2"))
            if stride > 1:
                o = avgpool2(o, stride)
            o = bn(conv2d(o, sd[p + "conv3.weight"]), p + "bn3")
            if p + "downsample.0.weight" in sd:
                skip = avgpool2(h, stride) if stride > 1 else h
                skip = bn(conv2d(skip, sd[p + "downsample.0.weight"]), p + "downsample.1")
            else:
                skip = h
            h = relu(o + skip)
    return attnpool(h, sd, "attnpool.", heads), stats


def triplet_margin_loss(a, p, n, margin=0.2, eps=1e-6):
    dap = np.sqrt((((a - p) + eps) ** 2).sum(1))
    dan = np.sqrt((((a - n) + eps) ** 2).sum(1))
    return np.maximum(margin + dap - dan, 0).mean()


def adam_step(param, grad, m, v, step, lr=1e-5, wd=0.002, b1=0.9, b2=0.999, eps=1e-8):
    g = grad + wd * param
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    param = param - (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + eps)
    return param, m, v
