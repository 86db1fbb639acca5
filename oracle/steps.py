"""The triplet training step and embedding pass on CPU (TEST ORACLE).

Follows /root/reference/train.py:
  get_loss           train.py:27-37  (three separate forwards -> BN stats per branch)
  triplet_train step train.py:59-70  (zero_grad, backward, Adam.step)
  optimizer          train.py:158    (Adam(lr, weight_decay) — coupled L2)
  loss               train.py:169    (nn.TripletMarginLoss(margin=utils.MARGIN=0.2))
and inference.py:72-92 (eval-mode gallery embedding).
"""
from __future__ import annotations

import torch
from torch import nn

from . import encoder

MARGIN = 0.2  # utils.py:77


def build(layers, output_dim, heads, res, width, seed=1234, with_classification=False, **kw):
    cls = encoder.ModifiedResNet_with_classification if with_classification else encoder.ModifiedResNet
    m = cls(layers, output_dim, heads=heads, input_resolution=res, width=width, **kw)
    encoder.init_params(m, seed)
    return m


def get_loss(loss_fn, model, elements):
    """train.py:27-37 dispatch on the arity of the model output."""
    s, p, n = (model(e) for e in elements[:3])
    if isinstance(s, torch.Tensor):
        return loss_fn(s, p, n), (s, p, n)
    if len(s) == 2:
        return loss_fn(s[0], p[0], n[0], s[1], p[1], elements[3]), (s[0], p[0], n[0])
    return loss_fn(s[0], p[0], n[0], s[1], p[1], s[2], p[2], elements[3], elements[4]), (s[0], p[0], n[0])


def train_step(model, optimizer, loss_fn, elements):
    """One iteration of train.py:59-70; returns (loss, embeddings) detached."""
    model.train()
    loss, embs = get_loss(loss_fn, model, elements)
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return loss.detach(), tuple(e.detach() for e in embs)


def make_optimizer(model, lr=1e-5, weight_decay=0.002):
    return torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)


def make_loss(margin=MARGIN):
    return nn.TripletMarginLoss(margin=margin)


@torch.no_grad()
def embed(model, images, batch=50):
    """inference.py:72-92: eval mode, batches of 50, concatenated features."""
    model.eval()
    feats = [model(images[i:i + batch]) for i in range(0, len(images), batch)]
    return torch.cat([f if isinstance(f, torch.Tensor) else f[0] for f in feats])
