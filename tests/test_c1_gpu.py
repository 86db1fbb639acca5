"""Configuration C1 (BASELINE.json configs[0]): the "ResNet18"
encoder ModifiedResNet((2,2,2,2), output_dim=128) at 224x224, width 64, on the
HIP path against the CPU oracle (/root/reference/train.py:59-70 step,
models.py:284-360 model), at a small batch (4 triplets) so the float64
backward takes seconds; plus the train.py CLI at the reference's default batch
of 32 (train.py:108) on that model.

The checks are test_c2_gpu.py's (same damped weights and bars): f32 mode
embeddings within 1e-3, loss, every gradient (mask-conditioned), BN running
statistics and the eval embedding; bf16 mode relative-L2 bars against PyTorch's
own bf16 autocast."""
import pytest
import torch

from test_c2_gpu import check_bf16_step, check_f32_step, oracle_runs

pytestmark = pytest.mark.gpu

C1 = dict(layers=(2, 2, 2, 2), output_dim=128, heads=32, res=224, width=64)


@pytest.fixture(scope="module")
def oracle_c1():
    return oracle_runs(C1)


def test_c1_f32_step_matches_oracle(oracle_c1, dev):
    check_f32_step(oracle_c1, dev, "C1")


def test_c1_bf16_step_accuracy(oracle_c1, dev):
    check_bf16_step(oracle_c1, dev, False, "C1")


def test_c1_train_cli_batch32(tmp_path, dev, monkeypatch):
    """train.py -b 32 on the C1 model (synthetic 224x224 triplets, one epoch of
    64 triplets = two steps), then the inference pass: finite losses, results
    and the model file written as the reference does"""
    import train
    monkeypatch.chdir(tmp_path)
    training, inf = train.main(["--layers", "2,2,2,2", "--output_dim", "128", "-b", "32", "--synthetic_n", "64",
                                "-e", "1", "--dtype", "bf16", "--inference"])
    losses = training["train_losses"]
    assert len(losses) == 1 and torch.isfinite(torch.tensor(losses)).all(), losses
    assert inf["count"] == inf["size"] and inf["size"] > 0
    assert 1 <= inf["min"] <= inf["max"] <= inf["size"]
    assert any((tmp_path / "models").glob("ModifiedResNet_*.pth"))
