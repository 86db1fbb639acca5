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


def _rccl_entry(port, q):
    """one rank over RCCL ("nccl" on ROCm) on the real device: the process group,
    the overlapped bucketed all-reduce on its comm stream, the buffer broadcast,
    the coalesced all-reduce of the ViT path and the sharded retrieval's
    collectives all run through RCCL (at world size 1 every collective is an
    identity, so the results must equal the plain single-process ones)"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
                      ARTSBIR_DDP_WORLD1="1")
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "art-sbir_amd"))
    sys.path.insert(0, root)
    import ddp
    ddp.init_distributed()
    try:
        import engine
        import knn
        import losses
        import models
        import numpy as np
        from oracle import retrieval as oret
        assert dist.get_backend() == "nccl"
        engine.set_deterministic(True)
        dev = torch.device("cuda", 0)
        torch.manual_seed(6)
        model = models.ModifiedResNet((1, 2, 1, 1), 32, heads=8, input_resolution=64, width=16).to(dev)
        model.compute_dtype = torch.float32
        model.train()
        loss_fn = losses.TripletMarginLoss(margin=0.2)
        g = torch.Generator(device=dev).manual_seed(41)
        xs = [torch.randn(4, 3, 64, 64, device=dev, generator=g) + i for i in range(3)]
        state = {k: v.clone() for k, v in model.state_dict().items()}
        want = _grads(model, loss_fn, xs)
        model.load_state_dict(state)
        ddp.broadcast_buffers(model)
        reducer = ddp.attach_overlapped_reducer(model, bucket_bytes=64 << 10)
        _grads(model, loss_fn, xs)
        n_during = reducer.launched_before_end
        reducer.finish()
        torch.cuda.synchronize()
        got = model._hip_engine._grads.flat
        err = float((got - want).abs().max()) / float(want.abs().max())
        ts = [torch.randn(1000, device=dev), torch.randn(37, device=dev)]
        before = [t.clone() for t in ts]
        ddp.allreduce_tensors(ts)
        vit_ok = all(torch.equal(a, b) for a, b in zip(ts, before))
        gal, qs, pos = oret.synthetic_gallery(3000, 64, 20, noise=1.5)
        idx, _, rank = knn.knn_sharded(torch.from_numpy(qs).to(dev), torch.from_numpy(gal).to(dev), 0, 10,
                                       torch.from_numpy(pos).to(dev))
        ri = np.array([oret.topk(oret.distances(q, gal), 10)[0] for q in qs])
        rr = np.array([oret.rank_of(oret.distances(qs[i], gal), pos[i]) for i in range(len(qs))])
        knn_ok = bool((idx.cpu().numpy() == ri).all() and (rank.cpu().numpy() == rr).all())
        q.put((err, n_during, vit_ok, knn_ok))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_collectives():
    """RCCL initialised on the MI355X (the 8-GPU C3 run is the driver's; one
    rank here) through the same ddp.py / knn.py code bench.py and train.py use"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_entry, args=(_free_port(), q))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0, p.exitcode
    err, n_during, vit_ok, knn_ok = q.get(timeout=5)
    print(f"RCCL world 1: gradient max rel diff {err:.2e}, all-reduces inside the backward {n_during}")
    assert err < 1e-5, err  # the f32 atomics of the weight gradients add in a different order per run
    assert n_during >= 3
    assert vit_ok and knn_ok
