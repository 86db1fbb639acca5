"""GPU preprocessing (csrc/preprocess.hip via preprocess.ClipPreprocess) against
the CPU transform of the reference (models.py:289-295: torchvision Resize
BICUBIC -> CenterCrop -> RGB -> ToTensor -> Normalize, which runs Pillow's
resampling; models.ClipTransform restates it with Pillow directly — torchvision
is not installed here, so the Pillow/torch steps themselves are the oracle).
The bar is bit-identical f32 output."""
import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu

SIZES = [(300, 200), (224, 224), (100, 150), (1024, 513), (225, 224), (224, 225), (50, 50), (640, 480), (97, 331),
         (2000, 1500)]


def _images(seed):
    rng = np.random.default_rng(seed)
    out = []
    for i, (w, h) in enumerate(SIZES):
        mode = "L" if i % 3 == 2 else "RGB"
        shape = (h, w) if mode == "L" else (h, w, 3)
        # smooth content plus noise: exercises both flat regions and overshoot clipping
        base = rng.integers(0, 256, size=shape, dtype=np.uint8)
        if i % 2:
            yy, xx = np.mgrid[0:h, 0:w]
            grad = ((xx * 255) // max(w - 1, 1)).astype(np.uint8)
            base = grad if mode == "L" else np.repeat(grad[..., None], 3, axis=2)
            base[::7, ::5] = 255 - base[::7, ::5]
        out.append(Image.fromarray(base, mode))
    return out


@pytest.mark.parametrize("res", [224, 64])
def test_gpu_preprocess_bit_identical_to_pillow_transform(res, dev):
    import models
    import preprocess
    imgs = _images(res)
    gpu = preprocess.ClipPreprocess(res, device=dev)(imgs).cpu()
    ref = models.ClipTransform(res)
    for i, im in enumerate(imgs):
        want = ref(im)
        assert gpu[i].shape == want.shape
        diff = (gpu[i] != want).sum().item()
        assert diff == 0, (im.size, im.mode, diff, (gpu[i] - want).abs().max().item())


def test_gpu_preprocess_rejects_other_modes(dev):
    import preprocess
    with pytest.raises(NotImplementedError):
        preprocess.ClipPreprocess(32, device=dev)([Image.new("P", (40, 40))])
    assert preprocess.ClipPreprocess(32, device=dev)([]).shape == (0, 3, 32, 32)


def _pil_sketch_pipeline(img, ops, boxes, res):
    """the reference's sketch transform for given random draws, on Pillow / torch
    (transformations.py:18-34: Resize((res, res), BICUBIC), RGB, the warps through
    Image.transform as torchvision's PIL backend calls it, ToTensor, erasing, Normalize)"""
    import models
    im = img.resize((res, res), Image.BICUBIC) if img.size != (res, res) else img
    im = im.convert("RGB")
    for what, co in ops:
        if what == "perspective":
            im = im.transform(im.size, Image.PERSPECTIVE, co, Image.BILINEAR, fillcolor=(255, 255, 255))
        else:
            im = im.transform(im.size, Image.AFFINE, co, Image.NEAREST, fillcolor=(255, 255, 255))
    t = torch.from_numpy(np.asarray(im, dtype=np.float32).copy() / 255.0).permute(2, 0, 1).contiguous()
    for i, j, h, w in boxes:
        t[:, i:i + h, j:j + w] = 1.0
    mean = torch.tensor(models.CLIP_MEAN)[:, None, None]
    std = torch.tensor(models.CLIP_STD)[:, None, None]
    return (t - mean) / std


@pytest.mark.parametrize("version", ["V1", "V2"])
def test_gpu_sketch_augmentation_bit_identical_to_pillow(version, dev):
    import preprocess
    res = 224
    imgs = _images(7)[:8]
    g = torch.Generator().manual_seed(123)
    aug = preprocess.SketchAugment(version, res, device=dev, generator=g)
    got = aug(imgs).cpu()
    g2 = torch.Generator().manual_seed(123)  # the same draws again, for the Pillow pipeline
    plans = [preprocess.sample_sketch_ops(aug.cfg, res, res, g2) for _ in imgs]
    kinds = set()
    for i, (im, (ops, boxes)) in enumerate(zip(imgs, plans)):
        kinds |= {w if w == "perspective" else preprocess._affine_kind(c) for w, c in ops}
        want = _pil_sketch_pipeline(im, ops, boxes, res)
        diff = (got[i] != want).sum().item()
        assert diff == 0, (i, [w for w, _ in ops], boxes, diff)
    assert {"perspective", 1, 2} <= kinds  # every warp kind was exercised


def test_gpu_warp_kinds_against_pillow(dev):
    """each warp kind alone, at parameters beyond the random ranges (large shear,
    strong perspective, scale-down), against Image.transform"""
    import preprocess
    res = 96
    rng = np.random.default_rng(5)
    src = Image.fromarray(rng.integers(0, 256, (res, res, 3), dtype=np.uint8))
    cases = [("affine", preprocess.inverse_affine_matrix([48.0, 48.0], 0.0, [0, 0], 0.7, [0.0, 0.0])),
             ("affine", preprocess.inverse_affine_matrix([48.0, 48.0], 33.0, [5, -9], 1.4, [20.0, -12.0])),
             ("perspective", preprocess.perspective_coeffs([[0, 0], [95, 0], [95, 95], [0, 95]],
                                                           [[20, 5], [70, 18], [90, 80], [3, 60]]))]
    aug = preprocess.SketchAugment("V1", res, device=dev)
    rgb = torch.from_numpy(np.asarray(src).copy())[None].to(dev)
    for what, co in cases:
        got = aug.apply(rgb, [([(what, co)], [])]).cpu()[0]
        want = _pil_sketch_pipeline(src, [(what, co)], [], res)
        assert (got != want).sum().item() == 0, what


def test_gpu_data_path_matches_cpu_transform_path(dev):
    """train.py's input pipeline with --gpu_preprocess (DataLoader workers only
    decode, one ClipPreprocess call per branch) gives bit-identically the batch
    of the reference's pipeline (the model transform in the workers,
    train.py:152-155) on the same decoded images, sketches (grayscale, 256^2) and
    photos (RGB, ragged 256..640 px) alike"""
    import random

    import data_preparation
    import models
    import train
    from torch.utils.data import DataLoader
    res = 224
    tr = models.ClipTransform(res)
    gpu_ds, _ = data_preparation.get_datasets("Synthetic", n=40, resolution=res, decode_only=True, transform=tr)
    cpu_ds, _ = data_preparation.get_datasets("Synthetic", n=40, resolution=res, pixels=True, transform=tr)
    model = types_ns(res)
    random.seed(9)
    gb = next(iter(DataLoader(gpu_ds, batch_size=12, collate_fn=data_preparation.collate_decoded)))
    random.seed(9)
    cb = next(iter(DataLoader(cpu_ds, batch_size=12)))
    g = train._to_device(gb, model)
    c = [t.to(dev) for t in cb]
    for x, y in zip(g, c):
        assert x.shape == y.shape == (12, 3, res, res)
        assert torch.equal(x, y), (x - y).abs().max().item()


def types_ns(res):
    import types
    return types.SimpleNamespace(input_resolution=res)


def test_train_cli_gpu_preprocess(tmp_path, dev, monkeypatch):
    """train.py --gpu_preprocess --inference end to end (gallery embedding and
    sketch queries through the GPU transform too)"""
    import train
    monkeypatch.chdir(tmp_path)
    training, inf = train.main(["--layers", "1,1,1,1", "--width", "16", "--resolution", "64", "--output_dim", "32",
                                "-b", "4", "--synthetic_n", "40", "-e", "1", "--inference", "--dtype", "bf16",
                                "--gpu_preprocess", "--no_save"])
    assert training["train_losses"][0] == training["train_losses"][0]
    assert inf["size"] == 4 and inf["count"] == 4
