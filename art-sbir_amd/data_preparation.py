"""Datasets feeding the hot path (/root/reference/data_preparation.py, hot-path parts).

  InferenceDataset      data_preparation.py:24-41 — gallery paths de-duplicated
                        (first occurrence kept) and SORTED; this order defines the
                        gallery index used by retrieval ranks.
  SyntheticTripletDataset  stands in for the Sketchy/Kaggle datasets (no data and
                        no network here): same interface as RetrievalDataset
                        (sketch_paths, photo_paths, __getitem__ -> (sketch, pos,
                        neg) with the negative drawn by random.choice after
                        random.seed(seed), state_dict), sketch names
                        "<photo-stem>-<n>.png" so inference.py's name parsing and
                        utils.find_image_index work unchanged.  Images are
                        generated deterministically from the path (PCG64 seeded
                        by crc32(path)): photos uniform [0,1), sketches 90 % white
                        / 10 % black strokes correlated with their photo, both
                        through the CLIP normalize of models.py:294.
  SyntheticKaggleInferenceDataset  stands in for KaggleInferenceDatasetV1
                        (data_preparation.py:696-722): sketches only ("data/kaggle/
                        <sketch_type>/<photo-stem>-k<n>.png", every tenth one for a
                        photo outside the gallery), __getitem__ -> [sketch]
  get_datasets          data_preparation.py:796-848 factory ("Synthetic*" — the name
                        may carry "Kaggle" / "Mixed", which selects the reference's
                        Kaggle/Mixed behaviour downstream — and "KaggleInferenceV1").
"""
from __future__ import annotations

import random
import zlib
from pathlib import Path
from typing import Dict, List

import numpy as np
import torch
from torch.utils.data import Dataset

MEAN = np.array((0.48145466, 0.4578275, 0.40821073), np.float32)[:, None, None]
STD = np.array((0.26862954, 0.26130258, 0.27577711), np.float32)[:, None, None]


def _rng(path) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(zlib.crc32(str(path).encode())))


def synthetic_photo(path, res: int) -> torch.Tensor:
    img = _rng(path).random((3, res, res), dtype=np.float32)
    return torch.from_numpy((img - MEAN) / STD)


def synthetic_sketch(path, photo_path, res: int) -> torch.Tensor:
    # strokes where the photo's luminance is low, plus 5 % noise: a learnable pairing
    photo = _rng(photo_path).random((3, res, res), dtype=np.float32).mean(0)
    noise = _rng(path).random((res, res), dtype=np.float32)
    stroke = (photo < 0.3) ^ (noise < 0.05)
    img = np.where(stroke, 0.0, 1.0).astype(np.float32)[None].repeat(3, axis=0)
    return torch.from_numpy((img - MEAN) / STD)


# ---------------------------------------------------------------- pixel mode
# The reference's datasets open image FILES (PIL) and run the model's transform
# (models.py:289-295) in DataLoader workers (train.py:154-155).  Pixel mode
# reproduces that input pipeline: an image is the decoded file when it exists,
# else a deterministic stand-in of the same kind (a decoded photo of 256..640 px
# per side, RGB; a 256 x 256 grayscale sketch, like Sketchy's PNGs), and then
#   decode_only=False  the CPU transform (PIL resize / crop / normalise), as the reference;
#   decode_only=True   the uint8 pixels only: the GPU transform runs on the whole
#                      batch in one library call (preprocess.ClipPreprocess,
#                      SURVEY §8f row 3), so the workers only decode.

def synthetic_pixels(path, kind: str) -> np.ndarray:
    rng = _rng(path)
    if kind == "sketch":
        img = np.full((256, 256), 255, np.uint8)
        img[rng.random((256, 256)) < 0.1] = 0
        return img
    w, h = (int(v) for v in rng.integers(256, 641, size=2))
    base = rng.integers(0, 256, size=(h // 8 + 1, w // 8 + 1, 3), dtype=np.uint8)  # blocky content plus noise
    img = np.repeat(np.repeat(base, 8, axis=0), 8, axis=1)[:h, :w]
    return np.ascontiguousarray(img ^ rng.integers(0, 32, size=(h, w, 3), dtype=np.uint8))


def load_pixels(path, kind: str) -> np.ndarray:
    """the decoded image file (HxW 'L' or HxWx3 'RGB' uint8), or its stand-in"""
    if Path(path).is_file():
        from PIL import Image
        with Image.open(path) as im:
            if im.mode not in ("L", "RGB"):
                im = im.convert("RGB")
            return np.asarray(im).copy()
    return synthetic_pixels(path, kind)


def pixels_item(path, kind, transform, decode_only):
    a = load_pixels(path, kind)
    if decode_only:
        return torch.from_numpy(a)
    from PIL import Image
    return transform(Image.fromarray(a))


def collate_decoded(batch):
    """DataLoader collate for decode-only items: ragged uint8 images stay lists
    (one list per element of the item), everything else is stacked as usual"""
    from torch.utils.data import default_collate
    if isinstance(batch[0], torch.Tensor):
        return list(batch) if batch[0].dtype == torch.uint8 else default_collate(batch)
    return [collate_decoded([b[i] for b in batch]) for i in range(len(batch[0]))]


class InferenceDataset(Dataset):
    def __init__(self, image_paths: List[Path], transform=None, resolution: int = 224, pixels: bool = False,
                 decode_only: bool = False):
        super().__init__()
        self.transform = transform
        self.resolution = resolution
        self.pixels, self.decode_only = pixels or decode_only, decode_only
        self.image_paths = list(dict.fromkeys(image_paths))
        self.image_paths.sort()

    def __len__(self) -> int:
        return len(self.image_paths)

    def __getitem__(self, idx: int) -> torch.Tensor:
        p = self.image_paths[idx]
        if self.pixels:
            return pixels_item(p, "photo", self.transform, self.decode_only)
        if Path(p).is_file() and self.transform is not None:
            from PIL import Image
            return self.transform(Image.open(p))
        return synthetic_photo(p, self.resolution)


class SyntheticTripletDataset(Dataset):
    def __init__(self, n: int = 256, resolution: int = 224, mode: str = "train", split_ratio: float = 0.1,
                 size: float = 1.0, seed: int = 42, transform=None, dups: int = 1, name: str = None,
                 pixels: bool = False, decode_only: bool = False):
        super().__init__()
        self.pixels, self.decode_only = pixels or decode_only, decode_only
        self.name = name or self.__class__.__name__
        if mode not in ("train", "test"):
            raise ValueError("invalid mode: [train, test]")
        random.seed(seed)
        self.mode, self.size, self.seed, self.split_ratio = mode, size, seed, split_ratio
        self.resolution, self.transform = resolution, transform
        total = max(2, int(n * size))
        n_test = max(1, int(round(total * split_ratio)))
        ids = list(range(total))
        ids = ids[n_test:] if mode == "train" else ids[:n_test]
        root = Path("data/synthetic")
        # several sketches per photo (Sketchy has ~5): "<stem>-<k>.png"
        self.photo_paths = [root / "photos" / f"img{i:07d}.jpg" for i in ids for _ in range(dups)]
        self.sketch_paths = [root / "sketches" / f"img{i:07d}-{k + 1}.png" for i in ids for k in range(dups)]

    def __len__(self) -> int:
        return len(self.sketch_paths)

    def load_image_sketch_tuple(self, idx):
        neg = random.choice(self.photo_paths)  # may pick the positive, as the reference does
        return self.sketch_paths[idx], self.photo_paths[idx], neg

    def __getitem__(self, idx):
        s, p, n = self.load_image_sketch_tuple(idx)
        if self.pixels:
            return tuple(pixels_item(x, k, self.transform, self.decode_only)
                         for x, k in ((s, "sketch"), (p, "photo"), (n, "photo")))
        r = self.resolution
        return synthetic_sketch(s, p, r), synthetic_photo(p, r), synthetic_photo(n, r)

    def sketch(self, idx):
        if self.pixels:
            return pixels_item(self.sketch_paths[idx], "sketch", self.transform, self.decode_only)
        return synthetic_sketch(self.sketch_paths[idx], self.photo_paths[idx], self.resolution)

    @property
    def state_dict(self) -> Dict:
        return {"dataset": self.name, "size": self.size, "img_number": len(self),
                "img_type": "synthetic", "img_format": "jpg", "sketch_format": "png", "seed": self.seed,
                "split_ratio": self.split_ratio, "mode": self.mode, "transform": str(self.transform)}


class SyntheticKaggleInferenceDataset(Dataset):
    def __init__(self, photo_paths: List[Path], sketch_type: str = 'sketches', sketch_format: str = 'png',
                 transform=None, resolution: int = 224, pixels: bool = False, decode_only: bool = False):
        super().__init__()
        self.pixels, self.decode_only = pixels or decode_only, decode_only
        self.sketch_type, self.sketch_format, self.transform = sketch_type, sketch_format, transform
        self.resolution = resolution
        root = Path("data/kaggle") / sketch_type
        photos = list(dict.fromkeys(photo_paths))
        self.sketch_paths, self.photo_of = [], []
        for i, p in enumerate(photos):
            stem = Path(p).stem if i % 10 != 9 else f"nogallery{i:05d}"
            self.sketch_paths.append(root / f"{stem}-k{i % 3 + 1}.{sketch_format}")
            self.photo_of.append(p)

    def __len__(self):
        return len(self.sketch_paths)

    def sketch(self, idx):
        if self.pixels:
            return pixels_item(self.sketch_paths[idx], "sketch", self.transform, self.decode_only)
        return synthetic_sketch(self.sketch_paths[idx], self.photo_of[idx], self.resolution)

    def __getitem__(self, idx):
        return [self.sketch(idx)]

    @property
    def state_dict(self):
        return {"dataset": "KaggleInferenceDatasetV1", "img_number": len(self), "sketch_type": self.sketch_type,
                "sketch_format": self.sketch_format, "transform": str(self.transform), "date": "synthetic"}


_LAST_TEST = [None]  # the gallery the Kaggle inference sketches refer to (the reference: data/kaggle on disk)


def get_datasets(dataset: str = "Synthetic", size: float = 1.0, sketch_format: str = 'png', img_format: str = 'jpg',
                 sketch_type: str = 'placeholder', img_type: str = 'photos', split_ratio: float = 0.1, seed: int = 42,
                 transform=None, n: int = 256, resolution: int = 224, pixels: bool = False, decode_only: bool = False,
                 **kw):
    """pixels / decode_only: pixel mode (see synthetic_pixels above)"""
    px = dict(pixels=pixels, decode_only=decode_only)
    if dataset.startswith("Synthetic"):
        name = None if dataset == "Synthetic" else dataset  # e.g. "SyntheticKaggleV1", "SyntheticMixedV1"
        tr = SyntheticTripletDataset(n, resolution, "train", split_ratio, size, seed, transform, name=name, **px)
        te = SyntheticTripletDataset(n, resolution, "test", split_ratio, size, seed, transform, name=name, **px)
        _LAST_TEST[0] = te
        return tr, te
    if dataset in ('KaggleInferenceV1', 'KaggleInferencedatasetV1'):
        te = _LAST_TEST[0] or SyntheticTripletDataset(n, resolution, "test", split_ratio, size, seed, transform)
        if not (pixels or decode_only):  # follow the gallery's mode
            px = dict(pixels=te.pixels, decode_only=te.decode_only)
        return None, SyntheticKaggleInferenceDataset(te.photo_paths, sketch_type, sketch_format, transform,
                                                     te.resolution, **px)
    raise Exception(f"{dataset} is not available (no datasets ship with this build; use Synthetic)")
