"""train.py / inference.py drop-in CLIs end to end on a tiny synthetic configuration."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

TINY = ["--layers", "1,1,1,1", "--width", "16", "--resolution", "64", "--output_dim", "32", "-b", "4",
        "--synthetic_n", "40", "-e", "1"]


def test_train_and_inference_cli(tmp_path, dev, monkeypatch):
    import train
    monkeypatch.chdir(tmp_path)
    training, inf = train.main(TINY + ["--inference", "--dtype", "bf16"])
    assert len(training["train_losses"]) == 1 and training["train_losses"][0] == training["train_losses"][0]
    for key in ("mean_reciprocal_rank", "size", "inference_time", "count", "mean", "std", "min", "25%", "50%", "75%",
                "max", "topk_acc", "retrieval_samples", "map@10", "image_features"):
        assert key in inf, key
    assert inf["count"] == 4 and inf["size"] == 4
    assert len(inf["topk_acc"]) == 10 and inf["topk_acc"][-1] == 1.0  # gallery of 4: every rank < 10
    # results written like the reference
    res = list((tmp_path / "results").iterdir())
    assert res and (res[0] / "inference.json").is_file()
    assert any((tmp_path / "models").glob("ModifiedResNet_SyntheticTripletDataset_*.pth"))
    feats = list((tmp_path / "data" / "image_features").iterdir())
    assert (feats[0] / "image_paths.csv").is_file() and (feats[0] / "image_features.csv").is_file()


def test_classification_model_step(dev):
    import losses
    import models
    import optim
    import utils
    m = models.ModifiedResNet_with_classification((1, 1, 1, 1), 32, heads=8, input_resolution=64, width=16,
                                                  num_classes=125).to(dev)
    m.train()
    x = torch.randn(4, 3, 64, 64, device=dev)
    feats, logits = m(x)
    assert feats.shape == (4, 32) and logits.shape == (4, 125)
    opt = optim.Adam(m.parameters(), lr=1e-4)
    loss_fn = utils.TripletMarginLoss_with_classification(margin=0.2)
    lab = torch.randint(0, 125, (4,), device=dev)
    outs = [m(torch.randn(4, 3, 64, 64, device=dev)) for _ in range(3)]
    loss = loss_fn(outs[0][0], outs[1][0], outs[2][0], outs[0][1], outs[1][1], lab)
    opt.zero_grad()
    loss.backward()
    assert m.classifier.weight.grad is not None and m.classifier.weight.grad.abs().sum() > 0
    assert m.conv1.weight.grad.abs().sum() > 0
    opt.step()


def test_kaggle_dataset_runs_second_inference_pass(tmp_path, dev, monkeypatch):
    """inference.py:154-163: a Kaggle / Mixed dataset is also ranked with the
    Kaggle inference sketches; the result nests both passes."""
    import train
    monkeypatch.chdir(tmp_path)
    _, inf = train.main(TINY + ["--inference", "--no_training", "-d", "SyntheticKaggle", "--no_save"])
    assert set(inf) == {"image_features", "drawing_stats", "sketch_stats"}
    first, second = inf["drawing_stats"], inf["sketch_stats"]
    assert first["size"] == second["size"] == 4
    assert first["count"] == 4 and second["count"] == 4
    assert 1 <= second["min"] <= second["max"] <= 4  # 1-based ranks within the 4-photo gallery
    assert second["inference_time"] >= first["inference_time"]
