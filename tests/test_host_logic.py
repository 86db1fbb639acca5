"""Host-side logic of the drop-in modules (no GPU): name parsing of
inference.py:33-37, the statistics of inference.py:116-134, dataset path
handling (data_preparation.py:16-51) and the feature cache round trip
(utils.py:258-284) — each checked against the oracle's restatement."""
import math
import os
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import retrieval as oret


def test_sketch_target_name_matches_oracle():
    import inference
    photos = [Path("data/x/photos/n02691156_10151.jpg")]
    art = [Path("data/x/artworks/starry.jpg")]
    cases = ["n02691156_10151-1.png", "n02691156_10151.png", "a-n02691156_10151-3.png", "a-b-c-d.png",
             "starry.png", "starry-2.png"]
    for s in cases:
        for paths in (photos, art):
            mine, ref = inference.sketch_target_name(Path("sk") / s, paths), oret.positive_name(Path("sk") / s, paths)
            if isinstance(ref, list):  # 4+ dash-separated parts: the reference never finds a positive
                assert mine is None, s
            else:
                assert mine == ref, s


def test_find_image_index():
    import utils
    paths = [Path("p/a.jpg"), Path("p/b.jpg"), Path("q/b.jpg")]
    assert utils.find_image_index(paths, "b") == 1
    assert utils.find_image_index(paths, "zz") == -1
    assert utils.find_image_index(paths, "b") == oret.find_image_index(paths, "b")


@pytest.mark.parametrize("ranks", [[0, 1, 2, 3, 9, 10, 57], [0], [4, 4, 4, 4], list(range(0, 400, 7))])
def test_retrieval_stats_match_oracle(ranks):
    import inference
    mine = inference.retrieval_stats(ranks, 10)
    ref = oret.metrics(ranks, 10)
    for k, v in ref.items():
        if isinstance(v, list):
            np.testing.assert_allclose(mine[k], v, rtol=1e-12)
        elif isinstance(v, float) and math.isnan(v):
            assert math.isnan(mine[k])
        else:
            assert mine[k] == pytest.approx(v, rel=1e-12), k


def test_pd_describe_empty_and_single():
    import inference
    assert inference.pd_describe([]) == {}
    d = inference.pd_describe([5])
    assert d["count"] == 1 and d["mean"] == 5 and math.isnan(d["std"])


def test_inference_dataset_dedups_and_sorts():
    import data_preparation
    paths = [Path("b.jpg"), Path("a.jpg"), Path("b.jpg"), Path("c.jpg")]
    ds = data_preparation.InferenceDataset(paths, resolution=32)
    assert ds.image_paths == oret.inference_dataset_paths(paths)
    assert len(ds) == 3 and tuple(ds[0].shape) == (3, 32, 32)
    # synthetic images are a pure function of the path
    assert torch.equal(ds[0], data_preparation.InferenceDataset([Path("a.jpg")], resolution=32)[0])


def test_synthetic_triplets_split_and_naming():
    import data_preparation
    import inference
    tr, te = data_preparation.get_datasets("Synthetic", n=40, resolution=32, split_ratio=0.1)
    assert len(tr) == 36 and len(te) == 4
    assert not set(tr.photo_paths) & set(te.photo_paths)
    for i in range(len(te)):
        # each sketch's positive is found by the inference name rule
        target = inference.sketch_target_name(te.sketch_paths[i], te.photo_paths)
        assert Path(te.photo_paths[i]).stem == target
    s, p, n = tr[0]
    assert s.shape == p.shape == n.shape == (3, 32, 32)
    with pytest.raises(Exception):
        data_preparation.get_datasets("SketchyV1")


def test_image_feature_cache_round_trip(tmp_path, monkeypatch):
    import data_preparation
    import utils
    monkeypatch.chdir(tmp_path)
    paths = [Path(f"img{i}.jpg") for i in range(5)]
    ds = data_preparation.InferenceDataset(paths, resolution=8)
    feats = torch.randn(5, 7)
    folder = utils.save_image_features("ModifiedResNet", "SyntheticTripletDataset", ds, feats)
    got_paths, got = utils.load_image_features(folder)  # utils.py:284 returns the folder name
    assert got_paths == ds.image_paths
    assert got.dtype == torch.float64 and torch.allclose(got.float(), feats)
    os.remove(Path("data/image_features") / folder / "image_features.npy")  # CSV-only cache (reference format)
    _, got2 = utils.load_image_features(folder)
    assert torch.allclose(got2.float(), feats, atol=1e-6)


def test_train_cli_keeps_reference_flags():
    import train
    a = train.parse_args(["-e", "2", "-b", "8", "-l", "1e-4", "-m", "none", "-d", "Synthetic", "-s", "0.5",
                          "--inference", "-w", "0.01", "--loss_type", "cosine", "--loss_margin", "0.3",
                          "--no_training", "--feature_folder", "ff"])
    assert (a.epochs, a.batch_size, a.learning_rate, a.dsize, a.weight_decay) == (2, 8, 1e-4, 0.5, 0.01)
    assert a.inference and a.no_training and a.loss_type == "cosine" and a.loss_margin == 0.3
    assert a.feature_folder == "ff"


def test_visualize_writes_reference_figures(tmp_path, monkeypatch):
    """visualization.visualize (visualization.py:262-273): the figure files of a
    one-pass and of a Kaggle/Mixed (nested) result, synthetic images rendered."""
    import data_preparation
    import visualization
    monkeypatch.chdir(tmp_path)
    _, te = data_preparation.get_datasets("Synthetic", n=40, resolution=32)
    photos = [str(p) for p in te.photo_paths]
    samples = [{str(te.sketch_paths[i]): [(p, 0.1 * j) for j, p in enumerate(photos)]} for i in range(2)]
    one = {"mean_reciprocal_rank": 0.5, "size": 4, "inference_time": 1.0, "topk_acc": [0.5] * 10,
           "retrieval_samples": samples}
    training = {"train_losses": [0.3, 0.2], "test_losses": [0.35, 0.25], "itrain_losses": [0.3], "itest_losses": [0.3],
                "iteration_loss_frequency": 312}
    visualization.visualize(tmp_path / "run1", training, one)
    for f in ("loss_curves", "loss_curves_iter", "retrieval_samples", "retrieval_samples_original", "topk_accuracy"):
        assert (tmp_path / "run1" / f"{f}.png").stat().st_size > 1000, f
    nested = {"image_features": "x", "drawing_stats": one, "sketch_stats": one}
    visualization.visualize(tmp_path / "run2", None, nested)
    for f in ("retrieval_samples_drawings", "retrieval_samples_sketches", "topk_accuracy_drawings",
              "topk_accuracy_sketches"):
        assert (tmp_path / "run2" / f"{f}.png").stat().st_size > 1000, f


def test_preprocess_plan_matches_torchvision_rules():
    """preprocess.plan: torchvision's resized size (shorter side -> res, int()
    of the long side) and centre-crop origin (round half to even)."""
    import preprocess
    assert preprocess.plan(300, 200, 224) == (336, 224, 56, 0)
    assert preprocess.plan(224, 225, 224) == (224, 225, 0, 0)   # (225-224)/2 = 0.5 -> 0
    assert preprocess.plan(224, 227, 224) == (224, 227, 0, 2)   # 1.5 -> 2
    assert preprocess.plan(97, 331, 224) == (224, 764, 0, 270)
    assert preprocess.plan(513, 1024, 224) == (224, 447, 0, 112)  # 111.5 -> 112


def test_pixel_mode_datasets_decode_only_and_cpu_transform():
    """pixel mode (SURVEY §8f row 3 data path): a decode-only item is the decoded
    uint8 image; the CPU-transform item is the model transform of exactly those
    pixels (models.py:289-295 through models.ClipTransform); ragged batches
    collate to lists"""
    import data_preparation
    import models
    from PIL import Image
    from torch.utils.data import DataLoader
    tr = models.ClipTransform(64)
    a, _ = data_preparation.get_datasets("Synthetic", n=20, resolution=64, decode_only=True)
    b, _ = data_preparation.get_datasets("Synthetic", n=20, resolution=64, pixels=True, transform=tr)
    assert a.pixels and a.decode_only and b.pixels and not b.decode_only
    import random
    random.seed(3)
    ia = a[2]
    random.seed(3)
    ib = b[2]
    assert ia[0].dtype == torch.uint8 and ia[0].shape == (256, 256)        # grayscale sketch
    assert ia[1].dtype == torch.uint8 and ia[1].ndim == 3 and ia[1].shape[2] == 3
    assert 256 <= ia[1].shape[0] <= 640 and 256 <= ia[1].shape[1] <= 640  # varied photo sizes
    for u8, t in zip(ia, ib):
        want = tr(Image.fromarray(u8.numpy()))
        assert torch.equal(t, want)
    shapes = {tuple(a[i][1].shape) for i in range(len(a))}
    assert len(shapes) > 1  # ragged
    batch = next(iter(DataLoader(a, batch_size=4, collate_fn=data_preparation.collate_decoded)))
    assert len(batch) == 3 and all(isinstance(x, list) and len(x) == 4 for x in batch)
    g = data_preparation.InferenceDataset(a.photo_paths, None, 64, decode_only=True)
    assert g[0].dtype == torch.uint8
