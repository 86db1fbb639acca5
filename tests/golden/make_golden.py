#!/usr/bin/env python3
"""Regenerate the golden fixtures of tests/golden from the CPU oracle.

    python tests/golden/make_golden.py

The reference publishes no golden vectors and may not be run here,
so these are produced by oracle/ (a CPU restatement of the reference path,
cross-pinned against an independent float64 numpy restatement).  Inputs are
generated from fixed PCG64 seeds; expected outputs are stored as summaries
(sum, L2 norm, 32 sampled entries at seeded positions) where full tensors would
bloat the repository.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import encoder as oenc  # noqa: E402
from oracle import retrieval as oret  # noqa: E402
from oracle import steps as osteps  # noqa: E402

TINY = dict(layers=(1, 1, 1, 1), output_dim=32, heads=8, res=64, width=16)
NSAMPLE = 32


def summary(t: torch.Tensor, key: str):
    a = t.detach().double().numpy().ravel()
    rng = np.random.Generator(np.random.PCG64(_stable_seed(key)))
    idx = rng.integers(0, a.size, size=min(NSAMPLE, a.size))
    return np.concatenate([[a.sum(), np.sqrt((a * a).sum())], a[idx]]), idx


def _stable_seed(key: str) -> int:
    import zlib
    return zlib.crc32(key.encode())


def encoder_fixture():
    torch.manual_seed(0)
    m = osteps.build(TINY["layers"], TINY["output_dim"], TINY["heads"], TINY["res"], TINY["width"], seed=1234)
    elements = list(oenc.synthetic_triplet(4, TINY["res"], seed=3))
    opt = osteps.make_optimizer(m, lr=1e-3, weight_decay=0.002)
    m.train()
    loss, embs = osteps.get_loss(osteps.make_loss(0.2), m, elements)
    opt.zero_grad()
    loss.backward()
    out = {"loss": np.array([loss.item()]), "emb_s": embs[0].detach().numpy(), "emb_p": embs[1].detach().numpy(),
           "emb_n": embs[2].detach().numpy()}
    for k, p in m.named_parameters():
        out["grad/" + k], _ = summary(p.grad, "grad/" + k)
    opt.step()
    for k, v in m.state_dict().items():
        if v.dtype.is_floating_point:
            out["state/" + k], _ = summary(v, "state/" + k)
        else:
            out["state/" + k] = v.numpy().reshape(-1).astype(np.int64)
    m.eval()
    with torch.no_grad():
        out["emb_eval"] = m(elements[0]).numpy()
    np.savez_compressed(os.path.join(HERE, "encoder_tiny.npz"), **out)


def golden_gallery():
    """the fixture's inputs (regenerated from seeds by the tests; not stored)."""
    g, qs, pos = oret.synthetic_gallery(4096, 64, 64, seed_g=11, seed_q=12)
    g[4000:4032] = g[0:32]      # exact duplicate rows -> distance ties
    qs[0:8] = g[0:8] + 1e-3     # queries whose positive has a duplicate
    pos = pos.copy()
    pos[60:] = -1               # queries without a positive
    return g, qs, pos


def retrieval_fixture():
    g, qs, pos = golden_gallery()
    idx, dist, ranks = [], [], []
    for i, q in enumerate(qs):
        d = oret.l2_distances(q, g)
        ti, td = oret.topk(d, 10)
        idx.append(ti)
        dist.append(td)
        ranks.append(oret.rank_of(d, pos[i]) if pos[i] >= 0 else len(g))
    metrics = oret.metrics([r for r, p in zip(ranks, pos) if p >= 0], 10)
    np.savez_compressed(os.path.join(HERE, "retrieval.npz"), positives=pos, topk_idx=np.array(idx),
                        topk_dist=np.array(dist), ranks=np.array(ranks), gallery_checksum=np.array([g.sum(), qs.sum()]))
    with open(os.path.join(HERE, "retrieval_metrics.json"), "w") as f:
        json.dump(metrics, f, indent=1, sort_keys=True)


def loss_adam_fixture():
    rng = np.random.Generator(np.random.PCG64(21))
    a, p, n = (torch.from_numpy(rng.standard_normal((16, 32), dtype=np.float32)).requires_grad_(True)
               for _ in range(3))
    loss = torch.nn.TripletMarginLoss(margin=0.2)(a, p, n)
    loss.backward()
    w = torch.from_numpy(rng.standard_normal((257,), dtype=np.float32)).requires_grad_(True)
    opt = torch.optim.Adam([w], lr=1e-3, weight_decay=0.002)
    grads = rng.standard_normal((3, 257), dtype=np.float32)
    w0 = w.detach().clone()
    for s in range(3):
        w.grad = torch.from_numpy(grads[s])
        opt.step()
    st = opt.state[w]
    np.savez_compressed(os.path.join(HERE, "loss_adam.npz"), a=a.detach().numpy(), p=p.detach().numpy(),
                        n=n.detach().numpy(), loss=np.array([loss.item()]), da=a.grad.numpy(), dp=p.grad.numpy(),
                        dn=n.grad.numpy(), w0=w0.numpy(), grads=grads, w3=w.detach().numpy(),
                        m3=st["exp_avg"].numpy(), v3=st["exp_avg_sq"].numpy())


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    encoder_fixture()
    retrieval_fixture()
    loss_adam_fixture()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
