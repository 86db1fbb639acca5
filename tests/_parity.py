"""Shared parity-test helpers (test infrastructure): the HIP forward's ReLU
decisions and the mask-conditioned oracle hook (oracle.encoder.RELU).

A ReLU network's gradient is piecewise linear in its inputs; an f32 forward
(HIP or PyTorch) differs from float64 by ~1e-7 relative, and the handful of
pre-activations within that distance of zero take the other branch ("flips").
Each flip moves one element's gradient contribution, which shows as a
percent-level error in a few small parameters.  Evaluating the float64 oracle
on the HIP forward's own ReLU decisions removes that noise, so a comparison
measures the kernels' arithmetic; the flips themselves are counted and bounded
(they may occur only where |x| is at f32 rounding distance from zero).
"""
import torch


def hip_relu_masks(m, elements, dev, batched=True):
    """the HIP forward's ReLU decisions, in the oracle's call order, per branch:
    [branch][relu] bool NCHW tensors (deterministic mode, a copy of the model so
    running statistics are untouched).  relu(bn(y)) > 0 exactly where bn(y) > 0
    (f32), so the stored activations / act_pool give the kernels' own masks.
    batched: one forward over all branches (forward_branches), else one forward
    per branch (separate model(x) calls)."""
    import copy
    import engine
    mc = copy.deepcopy(m)
    eng = mc._hip_engine
    eng.dtype = mc.compute_dtype
    mc.train()
    old = engine.set_deterministic(True)
    try:
        with torch.no_grad():
            if not batched:
                return [hip_relu_masks(mc, [e], dev)[0] for e in elements]
            _, ctx = eng.forward([e.to(dev) for e in elements], True, True)
            seq = []
            st = ctx["stem"]
            for y, bn in ((st["y1"], st["b1"]), (st["y2"], st["b2"]), (st["y3"], st["b3"])):
                seq.append(eng._act_pool(y, bn, 1, 0) > 0)
            for c in ctx["blocks"]:
                seq.append(c["a1"] > 0)
                seq.append(eng._act_pool(c["y2"], c["b2"], 1, 0) > 0)
                seq.append(c["out"] > 0)
    finally:
        engine.set_deterministic(old)
    G = len(elements)
    return [[t.permute(0, 3, 1, 2).cpu().chunk(G)[g] for t in seq] for g in range(G)]


class MaskFeed:
    """oracle.encoder.RELU hook: x * mask with the HIP masks, branch by branch, in
    forward order; records where the oracle's own decision (x > 0) differs"""

    def __init__(self, masks):
        self.masks = [list(b) for b in masks]
        self.branch, self.i = 0, 0
        self.flips, self.total, self.flip_mag = 0, 0, 0.0

    def __call__(self, x):
        mk = self.masks[self.branch][self.i]
        self.i += 1
        if self.i == len(self.masks[self.branch]):
            self.branch, self.i = self.branch + 1, 0
        own = x.detach() > 0
        diff = own != mk
        self.total += mk.numel()
        if diff.any():
            self.flips += int(diff.sum())
            scale = float(x.detach().abs().max())
            self.flip_mag = max(self.flip_mag, float(x.detach()[diff].abs().max()) / max(scale, 1e-30))
        return x * mk.to(x.dtype)




def conditioned_grads(build, elements, dt, masks):
    """loss and gradients of the oracle (build() -> a fresh oracle model) for one
    triplet step's three train-mode forwards, every ReLU replaced by the HIP
    masks; returns (loss, {name: grad f64}, MaskFeed)"""
    from oracle import encoder as oe
    from oracle import steps as osteps
    feed = MaskFeed(masks)
    oe.RELU = feed
    try:
        r = build().to(dt)
        r.train()
        loss, _ = osteps.get_loss(osteps.make_loss(0.2), r, [e.to(dt) for e in elements])
        loss.backward()
    finally:
        oe.RELU = None
    assert feed.branch == len(masks), "ReLU call order of the oracle and the HIP forward differ"
    return loss.item(), {k: p.grad.double() for k, p in r.named_parameters()}, feed


def max_rel_errors(grads, ref, noise, floor_frac=1e-4):
    """per parameter: (max |grads - ref|, max |noise - ref|) relative to max |ref|
    (floored at floor_frac x the largest gradient anywhere)"""
    floor = floor_frac * max(g.abs().max().item() for g in ref.values())
    out = {}
    for k, g in ref.items():
        scale = max(g.abs().max().item(), floor)
        out[k] = ((grads[k].double() - g).abs().max().item() / scale,
                  (noise[k].double() - g).abs().max().item() / scale)
    return out
