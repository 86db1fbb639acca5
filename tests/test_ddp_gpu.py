"""Data-parallel step with the gradient all-reduce overlapped with the backward
(ddp.OverlappedReducer driven by the engine's grad_hook), on
the real HIP engine: two ranks share the one GPU of the test box over gloo
(RCCL does not run two ranks on one device; the collective code path is the
same torch.distributed API).  Each rank trains on its own minibatch; after
finish() both must hold the average of the two single-process gradients
(train.py:59-70 per rank, averaged as torch DDP does)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _grads(model, loss_fn, xs):
    model.zero_grad(set_to_none=False)
    for p in model.parameters():
        if p.grad is not None:
            p.grad.zero_()
    out = model.forward_branches(xs)
    loss_fn(*out).backward()
    torch.cuda.synchronize()
    return model._hip_engine._grads.flat.clone()


def _entry(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "art-sbir_amd"))
    sys.path.insert(0, root)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import ddp
        import engine
        import losses
        import models
        engine.set_deterministic(True)  # same ReLU decisions in every run: differences are summation order only
        dev = torch.device("cuda", 0)
        torch.manual_seed(5)
        model = models.ModifiedResNet((1, 2, 1, 1), 32, heads=8, input_resolution=64, width=16).to(dev)
        model.compute_dtype = torch.float32
        model.train()
        loss_fn = losses.TripletMarginLoss(margin=0.2)
        batches = []
        for r in range(WORLD):
            g = torch.Generator(device=dev).manual_seed(40 + r)
            batches.append([torch.randn(4, 3, 64, 64, device=dev, generator=g) + i for i in range(3)])
        state = {k: v.clone() for k, v in model.state_dict().items()}
        single = []
        for r in range(WORLD):  # no hook attached: plain single-process gradients
            model.load_state_dict(state)
            single.append(_grads(model, loss_fn, batches[r]))
        want = sum(single) / WORLD
        model.load_state_dict(state)
        reducer = ddp.attach_overlapped_reducer(model, bucket_bytes=64 << 10)
        got = _grads(model, loss_fn, batches[rank])
        n_during = reducer.launched_before_end
        reducer.finish()
        torch.cuda.synchronize()
        got = model._hip_engine._grads.flat
        scale = want.abs().max().item()
        err = (got - want).abs().max().item() / scale
        q.put((rank, err, n_during, len(single[0]), float((single[0] - single[1]).abs().max()) / scale))
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_matches_averaged_gradients():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    assert codes == [0, 0], codes
    res = sorted(q.get(timeout=5) for _ in range(WORLD))
    for rank, err, n_during, n, diff in res:
        print(f"rank {rank}: max |avg - want| / max|want| = {err:.2e}, all-reduces launched inside "
              f"the backward: {n_during}, ranks' own gradients differ by {diff:.2e}")
        assert diff > 1e-3  # the two minibatches really give different gradients
        assert err < 1e-5, err
        assert n_during >= 3  # buckets went out during the backward, not only at finish()
