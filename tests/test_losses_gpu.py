"""Loss / head kernels vs torch fp32 CPU references of the same ops (utils.py:31-75, train.py:169-175)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _grads(fn, *xs):
    xs = [x.clone().requires_grad_(True) for x in xs]
    out = fn(*xs)
    out.backward(torch.ones_like(out))
    return out.detach(), [x.grad for x in xs]


@pytest.mark.parametrize("B,D", [(64, 128), (7, 33), (384, 512), (513, 768)])
def test_triplet_margin_loss(B, D, dev):
    """rows spread over B/4 workgroups (ragged last one), the mean in a fixed order"""
    import losses
    g = torch.Generator().manual_seed(0)
    a, p, n = (torch.randn(B, D, generator=g) for _ in range(3))
    ref, rg = _grads(torch.nn.TripletMarginLoss(margin=0.2), a, p, n)
    out, og = _grads(losses.TripletMarginLoss(margin=0.2), a.to(dev), p.to(dev), n.to(dev))
    assert torch.allclose(out.cpu(), ref, atol=1e-5)
    for x, y in zip(og, rg):
        assert torch.allclose(x.cpu(), y, atol=1e-6)


def test_cosine_triplet(dev):
    import losses
    import utils
    g = torch.Generator().manual_seed(1)
    a, p, n = (torch.randn(32, 64, generator=g) for _ in range(3))
    cos = lambda x, y: 1 - torch.nn.CosineSimilarity(dim=1)(x, y)  # noqa: E731
    ref, rg = _grads(torch.nn.TripletMarginWithDistanceLoss(distance_function=cos, margin=0.2), a, p, n)
    out, og = _grads(losses.TripletMarginWithDistanceLoss(distance_function=utils.cosine_distance, margin=0.2),
                     a.to(dev), p.to(dev), n.to(dev))
    assert torch.allclose(out.cpu(), ref, atol=1e-5)
    for x, y in zip(og, rg):
        assert torch.allclose(x.cpu(), y, atol=1e-5)


def test_cross_entropy_and_head(dev):
    import heads
    import losses
    g = torch.Generator().manual_seed(2)
    x = torch.randn(16, 96, generator=g)
    w = torch.randn(125, 96, generator=g) * 0.1
    b = torch.randn(125, generator=g) * 0.1
    lab = torch.randint(0, 125, (16,), generator=g)
    lab[3] = -100

    def ref_fn(x, w, b):
        return F.cross_entropy(F.linear(x, w, b), lab)

    def my_fn(x, w, b):
        return losses.CrossEntropyLoss()(heads.linear(x, w, b), lab.to(dev))
    ref, rg = _grads(ref_fn, x, w, b)
    out, og = _grads(my_fn, x.to(dev), w.to(dev), b.to(dev))
    assert torch.allclose(out.cpu(), ref, atol=1e-5)
    for a_, b_ in zip(og, rg):
        assert torch.allclose(a_.cpu(), b_, atol=1e-5)


def test_with_classification_losses(dev):
    import utils
    g = torch.Generator().manual_seed(3)
    s, p, n = (torch.randn(8, 32, generator=g) for _ in range(3))
    cs, cp = torch.randn(8, 70, generator=g), torch.randn(8, 70, generator=g)
    cs2, cp2 = torch.randn(8, 32, generator=g), torch.randn(8, 32, generator=g)
    l1, l2 = torch.randint(0, 70, (8,), generator=g), torch.randint(0, 32, (8,), generator=g)
    loss = utils.TripletMarginLoss_with_classification2(margin=0.2, classification_weight=0.25,
                                                        classification_weight2=0.5)
    out = loss(*(t.to(dev) for t in (s, p, n, cs, cp, cs2, cp2, l1, l2)))
    ref = (torch.nn.TripletMarginLoss(margin=0.2)(s, p, n) + 0.25 * (F.cross_entropy(cs, l1) + F.cross_entropy(cp, l1))
           + 0.5 * (F.cross_entropy(cs2, l2) + F.cross_entropy(cp2, l2)))
    assert abs(out.item() - ref.item()) < 1e-4
