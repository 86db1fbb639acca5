"""GPU image preprocessing: the encoder's transform
(/root/reference/models.py:289-295, torchvision Resize(res, BICUBIC) ->
CenterCrop(res) -> convert('RGB') -> ToTensor -> Normalize(CLIP)) for a batch
of decoded images in one library call (csrc/preprocess.hip), bit-identical to
the Pillow/torch CPU result of models.ClipTransform.

Decoding (JPEG/PNG) stays on the CPU with Pillow, as in the reference's
data loaders; the uint8 pixels go to the GPU once (pinned, asynchronous) and
the resampling, crop and normalisation run there.  Modes: 'L' and 'RGB' are
resampled as they are (grayscale becomes RGB afterwards, like convert('RGB'));
'P' / '1' (Pillow resizes them with NEAREST), 'RGBA' / 'LA' (premultiplied
resampling) and 16-bit modes are outside this kernel and raise.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import numpy as np
import torch

import _hip
from _hip import call

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def resized_size(w: int, h: int, res: int) -> Tuple[int, int]:
    """torchvision _compute_resized_output_size for an int size (shorter side -> res)"""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = res, int(res * long / short)
    return (new_short, new_long) if w <= h else (new_long, new_short)


def crop_origin(w: int, h: int, res: int) -> Tuple[int, int]:
    """torchvision center_crop offsets (Python round: half to even)"""
    return int(round((w - res) / 2.0)), int(round((h - res) / 2.0))


def plan(w: int, h: int, res: int) -> Tuple[int, int, int, int]:
    """(rw, rh, left, top) of one image"""
    rw, rh = resized_size(w, h, res)
    if rw < res or rh < res:
        raise NotImplementedError("CenterCrop padding (an image smaller than the crop after resizing)")
    left, top = crop_origin(rw, rh, res)
    return rw, rh, left, top


def _pixels(img) -> np.ndarray:
    """HxW (L) or HxWx3 (RGB) uint8 of a PIL image or array"""
    if hasattr(img, "mode"):
        if img.mode not in ("L", "RGB"):
            raise NotImplementedError(f"GPU preprocessing takes 'L' / 'RGB' images, got '{img.mode}'")
        a = np.asarray(img)
    else:
        a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim not in (2, 3) or (a.ndim == 3 and a.shape[2] not in (1, 3)):
        raise ValueError(f"expected HxW or HxWx3 uint8 pixels, got {a.dtype} {a.shape}")
    return np.ascontiguousarray(a)


class ClipPreprocess:
    """Batch transform on the GPU: ``ClipPreprocess(224)(images) -> [n,3,224,224] f32``"""

    def __init__(self, resolution: int = 224, mean=CLIP_MEAN, std=CLIP_STD, device="cuda"):
        self.resolution = resolution
        self.mean = (ctypes.c_float * 3)(*[float(np.float32(m)) for m in mean])
        self.std = (ctypes.c_float * 3)(*[float(np.float32(s)) for s in std])
        self.device = torch.device(device)

    def __call__(self, images: Sequence) -> torch.Tensor:
        res = self.resolution
        arrays = [_pixels(im) for im in images]
        n = len(arrays)
        out = torch.empty(n, 3, res, res, dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        # one pinned staging buffer for the batch, one host->device copy
        sizes = [a.nbytes for a in arrays]
        offs = np.concatenate([[0], np.cumsum([(s + 255) // 256 * 256 for s in sizes])]).astype(np.int64)
        host = torch.empty(int(offs[-1]), dtype=torch.uint8, pin_memory=True)
        hv = host.numpy()
        for a, o in zip(arrays, offs[:-1]):
            hv[o:o + a.nbytes] = a.reshape(-1)
        dev = host.to(self.device, non_blocking=True)
        descs = (_hip.ImageDesc * n)()
        for i, (a, o) in enumerate(zip(arrays, offs[:-1])):
            h, w = a.shape[:2]
            c = 1 if a.ndim == 2 else a.shape[2]
            rw, rh, left, top = plan(w, h, res)
            descs[i] = _hip.ImageDesc(dev.data_ptr() + int(o), h, w, c, w * c, rw, rh, left, top)
        ws_bytes = _hip.lib().artsbir_clip_preprocess_workspace(n, descs, res)
        if ws_bytes < 0:
            raise _hip.HipError(_hip.lib().artsbir_last_error().decode())
        ws = torch.empty(int(ws_bytes), dtype=torch.uint8, device=self.device)
        call("artsbir_clip_preprocess", n, descs, res, self.mean, self.std, out.data_ptr(), ws.data_ptr(), int(ws_bytes),
             _hip.stream())
        dev.record_stream(torch.cuda.current_stream(self.device))
        return out

    def __repr__(self):
        return f"ClipPreprocess(resize={self.resolution}, bicubic, center_crop, RGB, ToTensor, Normalize(CLIP), gpu)"
