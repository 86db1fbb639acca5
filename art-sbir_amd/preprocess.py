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
    if isinstance(img, torch.Tensor):
        a = img.detach().cpu().numpy()
    elif hasattr(img, "mode"):
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

    def stage(self, images: Sequence):
        """host pixels -> (device uint8 buffer, descriptors): one pinned staging
        buffer for the batch, one asynchronous host->device copy"""
        res = self.resolution
        arrays = [_pixels(im) for im in images]
        n = len(arrays)
        if n == 0:
            return None, (_hip.ImageDesc * 0)()
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
        return dev, descs

    def run(self, dev: torch.Tensor, descs, out: torch.Tensor | None = None, nbytes: float = 0.0) -> torch.Tensor:
        """the transform of images already in HBM (dev holds them, descs describes
        them): [n,3,res,res] f32 in one library call"""
        res = self.resolution
        n = len(descs)
        if out is None:
            out = torch.empty(n, 3, res, res, dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        ws_bytes = _hip.lib().artsbir_clip_preprocess_workspace(n, descs, res)
        if ws_bytes < 0:
            raise _hip.HipError(_hip.lib().artsbir_last_error().decode())
        ws = torch.empty(int(ws_bytes), dtype=torch.uint8, device=self.device)
        call("artsbir_clip_preprocess", n, descs, res, self.mean, self.std, out.data_ptr(), ws.data_ptr(), int(ws_bytes),
             _hip.stream(), kernel="clip_preprocess", nbytes=nbytes, tag=f"clip_preprocess n{n}")
        dev.record_stream(torch.cuda.current_stream(self.device))
        return out

    def __call__(self, images: Sequence) -> torch.Tensor:
        dev, descs = self.stage(images)
        return self.run(dev, descs)

    def __repr__(self):
        return f"ClipPreprocess(resize={self.resolution}, bicubic, center_crop, RGB, ToTensor, Normalize(CLIP), gpu)"


_PRE = {}


def clip_preprocessor(resolution: int = 224, device=None) -> ClipPreprocess:
    """the per-(resolution, device) ClipPreprocess of the data path (train.py /
    inference.py with --gpu_preprocess: DataLoader workers only decode)"""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (resolution, str(dev))
    if key not in _PRE:
        _PRE[key] = ClipPreprocess(resolution, device=dev)
    return _PRE[key]


def to_device_batch(batch, resolution: int, device=None):
    """a collated batch element -> a normalised [n,3,res,res] f32 tensor on the
    GPU: a list of decoded uint8 images goes through ClipPreprocess, a tensor
    (already transformed on the CPU) is just moved"""
    if isinstance(batch, (list, tuple)):
        return clip_preprocessor(resolution, device)(batch)
    return batch.to(device if device is not None else "cuda")


# ------------------------------------------------------------ augmentation
# transformations.py:18-56 — sketch_transformV1 / V2:
#   Resize((224, 224), BICUBIC) -> RGB
#   -> RandomApply(p1)[RandomPerspective(d, p=1, fill=255), RandomAffine(0, scale=(1.05, 1.3), fill=255)]
#   -> RandomApply(p2)[RandomAffine(deg, translate, scale, shear, fill=255)]
#   -> ToTensor -> RandomErasing(...) x k -> Normalize(CLIP)
# The random parameters are drawn with torch's generator in torchvision's own
# call order (RandomApply: torch.rand(1) > p skips; RandomPerspective:
# torch.rand(1) < p, then eight torch.randint; RandomAffine.get_params:
# uniform_ for angle, translate x / y, scale, shear x / y; RandomErasing:
# torch.rand(1) < p, then up to 10 tries of uniform_ area / exp(uniform_ log
# ratio) and two randint), so a seeded run draws what torchvision would draw
# (torchvision is not installed here: that equality is unpinned).  The pixel
# work — resize, the Pillow-exact warps and the erase/normalize — runs in
# libartsbir_hip (artsbir_resize_u8, artsbir_warp_u8, artsbir_erase_normalize).

import math

SKETCH_V1 = dict(p_geo=0.5, distortion=0.3, p_aff=0.5, degrees=15.0, translate=(0.1, 0.1), scale=(0.9, 1.1),
                 shear=(-7.0, 7.0, -7.0, 7.0), erasing=[(0.5, (0.05, 0.2), (0.3, 3.3))])
SKETCH_V2 = dict(p_geo=0.5, distortion=0.35, p_aff=0.7, degrees=15.0, translate=(0.3, 0.3), scale=(0.8, 1.2),
                 shear=(-10.0, 10.0, -10.0, 10.0),
                 erasing=[(0.7, (0.05, 0.1), (0.3, 3.3)), (0.7, (0.05, 0.1), (0.2, 2.0)), (0.7, (0.05, 0.1), (0.4, 4.0))])


def perspective_params(width, height, distortion_scale, g=None):
    """RandomPerspective.get_params"""
    hh, hw = height // 2, width // 2
    dw, dh = int(distortion_scale * hw), int(distortion_scale * hh)

    def ri(lo, hi):
        return int(torch.randint(lo, hi, size=(1,), generator=g).item())
    topleft = [ri(0, dw + 1), ri(0, dh + 1)]
    topright = [ri(width - dw - 1, width), ri(0, dh + 1)]
    botright = [ri(width - dw - 1, width), ri(height - dh - 1, height)]
    botleft = [ri(0, dw + 1), ri(height - dh - 1, height)]
    start = [[0, 0], [width - 1, 0], [width - 1, height - 1], [0, height - 1]]
    return start, [topleft, topright, botright, botleft]


def perspective_coeffs(startpoints, endpoints):
    """torchvision _get_perspective_coeffs: output -> input map, f64 lstsq rounded to f32"""
    a = torch.zeros(8, 8, dtype=torch.float64)
    for i, (p1, p2) in enumerate(zip(endpoints, startpoints)):
        a[2 * i, :] = torch.tensor([p1[0], p1[1], 1, 0, 0, 0, -p2[0] * p1[0], -p2[0] * p1[1]])
        a[2 * i + 1, :] = torch.tensor([0, 0, 0, p1[0], p1[1], 1, -p2[1] * p1[0], -p2[1] * p1[1]])
    b = torch.tensor(startpoints, dtype=torch.float64).view(8)
    return torch.linalg.lstsq(a, b, driver="gels").solution.to(torch.float32).tolist()


def affine_params(degrees, translate, scale_ranges, shears, img_size, g=None):
    """RandomAffine.get_params"""
    def uni(lo, hi):
        return float(torch.empty(1).uniform_(lo, hi, generator=g).item())
    angle = uni(float(degrees[0]), float(degrees[1]))
    if translate is not None:
        mdx, mdy = float(translate[0] * img_size[0]), float(translate[1] * img_size[1])
        tx = int(round(uni(-mdx, mdx)))
        ty = int(round(uni(-mdy, mdy)))
        tr = (tx, ty)
    else:
        tr = (0, 0)
    sc = uni(scale_ranges[0], scale_ranges[1]) if scale_ranges is not None else 1.0
    shx = shy = 0.0
    if shears is not None:
        shx = uni(shears[0], shears[1])
        if len(shears) == 4:
            shy = uni(shears[2], shears[3])
    return angle, tr, sc, (shx, shy)


def inverse_affine_matrix(center, angle, translate, scale, shear):
    """torchvision _get_inverse_affine_matrix (the output -> input map Pillow takes)"""
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m = [x / scale for x in m]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def erasing_params(img_h, img_w, scale, ratio, g=None):
    """RandomErasing.get_params (value given): (i, j, h, w) or None (no box in 10 tries)"""
    area = img_h * img_w
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        erase_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=g).item()
        aspect = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1], generator=g)).item()
        h = int(round(math.sqrt(erase_area * aspect)))
        w = int(round(math.sqrt(erase_area / aspect)))
        if not (h < img_h and w < img_w):
            continue
        i = int(torch.randint(0, img_h - h + 1, size=(1,), generator=g).item())
        j = int(torch.randint(0, img_w - w + 1, size=(1,), generator=g).item())
        return i, j, h, w
    return None


def _affine_kind(m):
    return 1 if (m[1] == 0 and m[3] == 0) else 2


def sample_sketch_ops(cfg, width, height, g=None):
    """the ordered pixel operations of one sketch (torchvision's draws, in order):
    [('perspective', coeffs) | ('affine', matrix)]*, [(i, j, h, w)]* erasing boxes"""
    ops = []
    if not (cfg["p_geo"] < torch.rand(1, generator=g).item()):  # RandomApply
        if torch.rand(1, generator=g).item() < 1.0:  # RandomPerspective(p=1)
            s, e = perspective_params(width, height, cfg["distortion"], g)
            ops.append(("perspective", perspective_coeffs(s, e)))
        ang, tr, sc, sh = affine_params((0.0, 0.0), None, (1.05, 1.3), None, [width, height], g)
        ops.append(("affine", inverse_affine_matrix([width * 0.5, height * 0.5], ang, list(tr), sc, list(sh))))
    if not (cfg["p_aff"] < torch.rand(1, generator=g).item()):
        d = cfg["degrees"]
        ang, tr, sc, sh = affine_params((-d, d), cfg["translate"], cfg["scale"], cfg["shear"], [width, height], g)
        ops.append(("affine", inverse_affine_matrix([width * 0.5, height * 0.5], ang, list(tr), sc, list(sh))))
    boxes = []
    for p, scale, ratio in cfg["erasing"]:
        if torch.rand(1, generator=g).item() < p:
            box = erasing_params(height, width, scale, ratio, g)
            if box is not None:
                boxes.append(box)
    return ops, boxes


class SketchAugment:
    """``SketchAugment('V1')(images) -> [n,3,224,224] f32`` on the GPU"""

    def __init__(self, version: str = "V1", resolution: int = 224, mean=CLIP_MEAN, std=CLIP_STD, device="cuda",
                 generator=None):
        self.cfg = SKETCH_V1 if version == "V1" else SKETCH_V2
        self.version, self.resolution, self.device, self.g = version, resolution, torch.device(device), generator
        self.mean = (ctypes.c_float * 3)(*[float(np.float32(m)) for m in mean])
        self.std = (ctypes.c_float * 3)(*[float(np.float32(s)) for s in std])

    def resize_u8(self, images) -> torch.Tensor:
        res = self.resolution
        arrays = [_pixels(im) for im in images]
        n = len(arrays)
        out = torch.empty(n, res, res, 3, dtype=torch.uint8, device=self.device)
        if n == 0:
            return out
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
            descs[i] = _hip.ImageDesc(dev.data_ptr() + int(o), h, w, c, w * c, res, res, 0, 0)  # Resize((res, res))
        ws_bytes = _hip.lib().artsbir_clip_preprocess_workspace(n, descs, res)
        if ws_bytes < 0:
            raise _hip.HipError(_hip.lib().artsbir_last_error().decode())
        ws = torch.empty(int(ws_bytes), dtype=torch.uint8, device=self.device)
        call("artsbir_resize_u8", n, descs, res, out.data_ptr(), ws.data_ptr(), int(ws_bytes), _hip.stream())
        dev.record_stream(torch.cuda.current_stream(self.device))
        return out

    def apply(self, rgb: torch.Tensor, plans) -> torch.Tensor:
        """rgb: [n,H,W,3] uint8 on the device; plans: sample_sketch_ops results"""
        n, H, W, _ = rgb.shape
        cur, nxt = rgb.contiguous(), torch.empty_like(rgb)
        steps = max((len(ops) for ops, _ in plans), default=0)
        ws = torch.empty(max(n, 1) * 256, dtype=torch.uint8, device=self.device)
        for k in range(steps):  # one batched launch per warp step; images with fewer steps copy
            descs = (_hip.WarpDesc * n)()
            for i, (ops, _) in enumerate(plans):
                d = descs[i]
                d.src, d.dst = cur[i].data_ptr(), nxt[i].data_ptr()
                d.fill[0] = d.fill[1] = d.fill[2] = 255
                if k < len(ops):
                    what, co = ops[k]
                    d.kind = 3 if what == "perspective" else _affine_kind(co)
                    for j, v in enumerate(co):
                        d.coeffs[j] = float(v)
                else:
                    d.kind = 0
            call("artsbir_warp_u8", n, descs, H, W, ws.data_ptr(), ws.numel(), _hip.stream())
            cur, nxt = nxt, cur
        out = torch.empty(n, 3, H, W, dtype=torch.float32, device=self.device)
        ed = (_hip.EraseDesc * n)()
        for i, (_, boxes) in enumerate(plans):
            e = ed[i]
            e.src = cur[i].data_ptr()
            e.nrect = len(boxes)
            for r, b in enumerate(boxes):
                for j in range(4):
                    e.rect[r][j] = int(b[j])
                e.value[r] = 1.0
        call("artsbir_erase_normalize", n, ed, H, W, self.mean, self.std, out.data_ptr(), ws.data_ptr(), ws.numel(),
             _hip.stream())
        return out

    def __call__(self, images):
        rgb = self.resize_u8(images)
        plans = [sample_sketch_ops(self.cfg, self.resolution, self.resolution, self.g) for _ in range(len(images))]
        return self.apply(rgb, plans)

    def __repr__(self):
        return f"SketchAugment({self.version}, {self.resolution}, gpu)"
