"""The drop-in CLI under torch.distributed.run on CPU (gloo, world_size 2):
train.main(... --inference) must return on BOTH ranks with the same inference
results (the reference calls inference.run_inference after training,
/root/reference/train.py:189; here that call is collective — sharded gallery
embedding + sharded retrieval — so every rank must take part), and only rank 0
writes the result files.  The encoder, loss, optimizer and the per-shard search
are CPU stand-ins (the HIP kernels need a GPU; tests/test_train_ddp_gpu.py runs
the real ones); what runs here is train.py / inference.py / ddp.py / knn.py's
own orchestration and collective code.

Also: rank-divergent BatchNorm running statistics must not make retrieval
depend on the world size (ddp.broadcast_buffers before the sharded embedding)."""
import functools
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_ddp_gloo import _cpu_local_search, _cpu_positive_keys

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _StandIn(torch.nn.Module):
    """CPU stand-in encoder with the attributes train.py uses and a BatchNorm
    (running statistics that diverge between ranks during training)"""

    def __init__(self, res, dim=8):
        super().__init__()
        torch.manual_seed(11)
        self.proj = torch.nn.Linear(3 * (res // 4) ** 2, dim)
        self.bn = torch.nn.BatchNorm1d(dim)
        self.transform = None
        self.trained_layers = []
        self.compute_dtype = torch.float32

    def freeze_layers(self):
        self.trained_layers.append('all')

    def forward(self, x):
        return self.bn(self.proj(torch.nn.functional.avg_pool2d(x, 4).flatten(1)))


def _patch_cpu(res):
    import inference
    import knn
    import optim
    import train
    import utils
    train.device = "cpu"
    inference.device = "cpu"
    utils.build_model = lambda *a, **k: _StandIn(res)
    train.make_loss = lambda *a, **k: torch.nn.TripletMarginLoss(margin=0.2)
    optim.Adam = torch.optim.Adam
    knn.knn_sharded = functools.partial(knn.knn_sharded, local_search=_cpu_local_search,
                                        positive_keys=_cpu_positive_keys,
                                        merge=lambda d, i, kk: knn.merge_topk(list(i), list(d), kk))


def _train_entry(rank, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD), RANK=str(rank),
                      LOCAL_RANK=str(rank), ARTSBIR_DIST_BACKEND="gloo")
    os.chdir(tmp)
    _patch_cpu(16)
    import train
    try:
        training, inf = train.main(["--resolution", "16", "--output_dim", "8", "-b", "4", "--synthetic_n", "60",
                                    "-e", "1", "--inference", "-d", "SyntheticKaggle"])
        q.put((rank, training["train_losses"], json.dumps(_strip(inf), sort_keys=True)))
    finally:
        dist.destroy_process_group()


def _strip(d):
    """inference dict without wall-clock fields"""
    if isinstance(d, dict):
        return {k: _strip(v) for k, v in d.items() if k != "inference_time"}
    return d


def test_train_main_inference_world2_returns_on_every_rank(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_entry, args=(r, port, str(tmp_path), q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    codes = [p.exitcode for p in procs]
    assert codes == [0, 0], codes
    res = sorted(q.get(timeout=5) for _ in range(WORLD))
    (_, l0, inf0), (_, l1, inf1) = res
    assert inf0 == inf1  # identical retrieval statistics on both ranks
    d = json.loads(inf0)
    assert set(d) == {"image_features", "drawing_stats", "sketch_stats"}  # Kaggle: the second pass ran too
    assert d["drawing_stats"]["size"] == 6 and d["drawing_stats"]["count"] == 6
    # only rank 0 wrote results / the model / the feature files
    assert len(list((tmp_path / "results").iterdir())) == 1
    assert len(list((tmp_path / "data" / "image_features").iterdir())) == 1


def _bn_entry(rank, port, tmp, q):
    """rank-divergent BN running statistics: sharded inference over 2 ranks must
    equal the 1-process inference of rank 0's model"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.chdir(tmp)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        _patch_cpu(16)
        import data_preparation
        import inference
        import knn
        from oracle import retrieval as oret
        model = _StandIn(16)
        model.bn.running_mean.fill_(0.3 * rank)  # as if each rank had trained on its own minibatches
        model.bn.running_var.fill_(1.0 + rank)
        _, test = data_preparation.get_datasets("Synthetic", n=130, resolution=16)
        out = inference.run_inference_sharded(model, test, "euclidean")
        # world-1 expectation with rank 0's statistics (mean 0, var 1)
        ref = _StandIn(16).eval()
        ids = data_preparation.InferenceDataset(test.photo_paths, None, 16)
        with torch.no_grad():
            g = torch.cat([ref(ids[i][None]) for i in range(len(ids))]).numpy()
            qs = torch.cat([ref(inference._Sketches(test)[i][None]) for i in range(len(test))]).numpy()
        pos = inference._positives(test, ids.image_paths)
        ranks = [oret.rank_of(oret.distances(qs[i], g, "euclidean"), pos[i]) for i in range(len(test))]
        want = inference.retrieval_stats(ranks, 10)
        ok = (out["mean_reciprocal_rank"] == pytest.approx(want["mean_reciprocal_rank"], rel=1e-12)
              and out["topk_acc"] == pytest.approx(want["topk_acc"]))
        q.put((rank, bool(ok), float(model.bn.running_mean[0])))
    finally:
        dist.destroy_process_group()


def test_sharded_inference_uses_rank0_bn_statistics(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_entry, args=(r, port, str(tmp_path), q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert [p.exitcode for p in procs] == [0, 0]
    res = sorted(q.get(timeout=5) for _ in range(WORLD))
    for rank, ok, rm in res:
        assert ok, rank
        assert rm == 0.0  # rank 1's running statistics were replaced by rank 0's


def _ff_entry(rank, port, tmp, q):
    """--feature_folder under two ranks: each rank reads the file, keeps its own
    row shard and the retrieval stays sharded (before, every rank ran the whole
    unsharded retrieval); results equal the run that wrote the features"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD), RANK=str(rank),
                      LOCAL_RANK=str(rank), ARTSBIR_DIST_BACKEND="gloo")
    os.chdir(tmp)
    _patch_cpu(16)
    import knn
    import train
    seen = []
    inner = knn.knn_sharded

    def spy(queries, shard, g_base, *a, **k):
        seen.append((int(shard.shape[0]), int(g_base)))
        return inner(queries, shard, g_base, *a, **k)
    knn.knn_sharded = spy
    try:
        args = ["--resolution", "16", "--output_dim", "8", "-b", "4", "--synthetic_n", "60", "-e", "1"]
        # both runs untrained (the seeded stand-in), so the queries are embedded by the same model
        _, inf = train.main(args + ["--inference", "--no_training", "--no_save"])
        folder = inf["image_features"]
        n_first = len(seen)
        _, inf2 = train.main(args + ["--inference", "--no_training", "--feature_folder", folder, "--no_save"])
        q.put((rank, json.dumps(_strip(inf), sort_keys=True), json.dumps(_strip(inf2), sort_keys=True),
               seen[n_first:]))
    finally:
        dist.destroy_process_group()


def test_feature_folder_inference_stays_sharded(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ff_entry, args=(r, port, str(tmp_path), q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert [p.exitcode for p in procs] == [0, 0]
    res = sorted(q.get(timeout=5) for _ in range(WORLD))
    (_, a0, b0, s0), (_, a1, b1, s1) = res
    assert b0 == b1  # same statistics on both ranks
    d_a, d_b = json.loads(a0), json.loads(b0)
    d_a.pop("image_features"), d_b.pop("image_features")
    assert d_a == d_b  # the file's features give the statistics the embedding run gave
    # each rank searched only its own contiguous shard of the gallery
    assert len(s0) == len(s1) == 1
    (n0, base0), (n1, base1) = s0[0], s1[0]
    assert base0 == 0 and base1 == n0 and n0 > 0 and n1 > 0
