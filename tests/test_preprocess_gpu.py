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
