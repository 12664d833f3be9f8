"""``dataset/transforms.py`` at the reference's module path (same names, arguments and semantics).

Two halves:

* **Box codecs** (transforms.py:26-83) — on the hot path: device tensors run the HIP kernel
  (csrc/codec.hip), CPU tensors the host path (``host.py``, the data-loader side).
* **Augmentation** (transforms.py:7-23, 86-383) — CPU work in DataLoader worker processes, as in the
  reference.  It draws from the module-level ``random`` stream in exactly the reference's order
  (``photometric_distort``'s shuffle and per-op draws first, then expand / crop / flip), so a seeded
  run produces the same boxes, labels and colour-op factors call for call
  (tests/test_transforms.py against fixtures made by running the reference's own ``transform``).
  ``random_crop``'s IoU is ``metrics.find_jaccard_overlap`` on CPU tensors, i.e. the drop-in's
  host path.  The reference's image operations are torchvision's functional ops on PIL images;
  torchvision is absent here, so they are rebuilt on PIL directly with torchvision's PIL-path
  definitions (hflip = FLIP_LEFT_RIGHT, resize = bilinear, brightness / contrast / saturation =
  ImageEnhance, hue = HSV shift with uint8 wrap-around, to_pil_image = ``mul(255).byte()``).  Pixel
  values are therefore "parity unpinned" (no torchvision to compare with); box arithmetic and the
  random stream are pinned.
"""
import random

import numpy as np
import torch
from PIL import Image, ImageEnhance

from .. import _lib as L
from .. import core
from .. import host
from .. import metrics
from ..metrics import on_host

IMAGENET_MEAN = [0.485, 0.456, 0.406]   # transforms.py:344-345
IMAGENET_STD = [0.229, 0.224, 0.225]


# ----------------------------------------------------------------------------- box codecs
def _rows(t, what):
    L.require_device(t, what=what)
    if t.dim() < 1 or t.shape[-1] != 4:
        raise RuntimeError('%s: expected [..., 4] boxes, got %s' % (what, tuple(t.shape)))
    return t.float()


def xy_to_cxcy(xy):
    """(x_min, y_min, x_max, y_max) -> (c_x, c_y, w, h)  (transforms.py:26-34)."""
    if on_host(xy):
        return host.xy_to_cxcy(xy)
    return core.codec('xy_to_cxcy', _rows(xy, 'xy_to_cxcy'))


def cxcy_to_xy(cxcy):
    """(c_x, c_y, w, h) -> (x_min, y_min, x_max, y_max)  (transforms.py:37-45)."""
    if on_host(cxcy):
        return host.cxcy_to_xy(cxcy)
    return core.codec('cxcy_to_xy', _rows(cxcy, 'cxcy_to_xy'))


def cxcy_to_gcxgcy(cxcy, priors_cxcy):
    """Encode w.r.t. priors: (c - pc) / (pwh / 10), log(wh / pwh) * 5  (transforms.py:48-66)."""
    if on_host(cxcy, priors_cxcy):
        return host.cxcy_to_gcxgcy(cxcy, priors_cxcy)
    return core.codec('encode_tenfive', _rows(cxcy, 'cxcy_to_gcxgcy'), priors_cxcy.float())


def gcxgcy_to_cxcy(gcxgcy, priors_cxcy):
    """Decode: g * pwh / 10 + pc, exp(g / 5) * pwh  (transforms.py:69-83)."""
    if on_host(gcxgcy, priors_cxcy):
        return host.gcxgcy_to_cxcy(gcxgcy, priors_cxcy)
    return core.codec('decode_tenfive', _rows(gcxgcy, 'gcxgcy_to_cxcy'), priors_cxcy.float())


# ----------------------------------------------------------------------------- image <-> tensor
def to_tensor(image):
    """PIL RGB -> float32 [3,H,W] = uint8 / 255 (torchvision ``to_tensor`` on a PIL image)."""
    a = np.asarray(image, dtype=np.uint8)
    return torch.from_numpy(a.astype(np.float32) / 255.0).permute(2, 0, 1).contiguous()


def to_pil(t):
    """float [3,H,W] -> PIL RGB by ``mul(255).byte()`` (truncation, as torchvision's
    ``to_pil_image`` converts float tensors)."""
    a = t.mul(255).byte().permute(1, 2, 0).contiguous().numpy()
    return Image.fromarray(a, mode='RGB')


def normalize(t, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    m = torch.tensor(mean, dtype=t.dtype).view(3, 1, 1)
    s = torch.tensor(std, dtype=t.dtype).view(3, 1, 1)
    return (t - m) / s


# ----------------------------------------------------------------------------- colour ops (PIL)
def adjust_brightness(image, factor):
    return ImageEnhance.Brightness(image).enhance(factor)


def adjust_contrast(image, factor):
    return ImageEnhance.Contrast(image).enhance(factor)


def adjust_saturation(image, factor):
    return ImageEnhance.Color(image).enhance(factor)


def adjust_hue(image, factor):
    """Shift the HSV hue channel by ``factor * 255`` with uint8 wrap-around (torchvision's PIL
    path; the float -> uint8 cast truncates toward zero, then wraps)."""
    if image.mode in ('L', '1', 'I', 'F'):
        return image
    h, s, v = image.convert('HSV').split()
    nh = np.asarray(h, dtype=np.uint8).copy()
    nh += np.uint8(int(factor * 255) % 256)
    return Image.merge('HSV', (Image.fromarray(nh, 'L'), s, v)).convert(image.mode)


# Looked up at call time (tests substitute recorders to compare the draw sequence).
DISTORTIONS = [adjust_brightness, adjust_contrast, adjust_saturation, adjust_hue]


# ----------------------------------------------------------------------------- augmentation
def decimate(tensor, m):
    """transforms.py:7-23: keep every m[d]-th index along each dimension d (None = keep all)."""
    assert tensor.dim() == len(m)
    for d in range(tensor.dim()):
        if m[d] is not None:
            tensor = tensor.index_select(dim=d, index=torch.arange(0, tensor.size(d), m[d]).long())
    return tensor


def expand(image, boxes, filler):
    """transforms.py:86-122: the [3,H,W] image placed at a random spot of a canvas up to 4x
    larger filled with ``filler``; pixel boxes shifted by the placement."""
    h, w = image.size(1), image.size(2)
    scale = random.uniform(1, 4)
    nh, nw = int(scale * h), int(scale * w)
    new_image = torch.tensor(filler, dtype=torch.float32).view(3, 1, 1).expand(3, nh, nw).clone()
    left = random.randint(0, nw - w)
    top = random.randint(0, nh - h)
    new_image[:, top:top + h, left:left + w] = image
    return new_image, boxes + torch.tensor([left, top, left, top], dtype=torch.float32)[None]


def random_crop(image, boxes, labels):
    """transforms.py:125-207: crop [3,H,W] with a minimum-overlap requirement drawn from
    {0, .1, .3, .5, .7, .9, None} (None = no crop), up to 50 trials per draw, sides in
    [0.3, 1] of the image, aspect in (0.5, 2); objects whose centres fall inside are kept and
    clipped."""
    h, w = image.size(1), image.size(2)
    while True:
        min_overlap = random.choice([0., .1, .3, .5, .7, .9, None])
        if min_overlap is None:
            return image, boxes, labels
        for _ in range(50):
            nh = int(random.uniform(0.3, 1) * h)
            nw = int(random.uniform(0.3, 1) * w)
            if not 0.5 < nh / nw < 2:
                continue
            left = random.randint(0, w - nw)
            top = random.randint(0, h - nh)
            crop = torch.tensor([left, top, left + nw, top + nh], dtype=torch.float32)
            overlap = metrics.find_jaccard_overlap(crop[None], boxes).squeeze(0)
            if overlap.max().item() < min_overlap:
                continue
            centers = (boxes[:, :2] + boxes[:, 2:]) / 2.
            inside = ((centers[:, 0] > left) & (centers[:, 0] < left + nw) &
                      (centers[:, 1] > top) & (centers[:, 1] < top + nh))
            if not inside.any():
                continue
            nb = boxes[inside, :]
            nb[:, :2] = torch.max(nb[:, :2], crop[:2]) - crop[:2]
            nb[:, 2:] = torch.min(nb[:, 2:], crop[2:]) - crop[:2]
            return image[:, top:top + nh, left:left + nw], nb, labels[inside]


def flip(image, boxes):
    """transforms.py:210-227: horizontal flip of a PIL image and its pixel boxes.  Like the
    reference, the x columns of ``boxes`` are rewritten in place before the column swap."""
    new_image = image.transpose(Image.FLIP_LEFT_RIGHT)
    boxes[:, 0] = image.width - boxes[:, 0] - 1
    boxes[:, 2] = image.width - boxes[:, 2] - 1
    return new_image, boxes[:, [2, 1, 0, 3]]


def resize(image, boxes, dims, return_percent_coords=True):
    """transforms.py:230-254: bilinear resize to dims = (H, W); boxes / (w, h, w, h) (fractional),
    or rescaled to the new pixel size."""
    new_image = image.resize((dims[1], dims[0]), Image.BILINEAR)
    old = torch.tensor([image.width, image.height, image.width, image.height], dtype=torch.float32)[None]
    new_boxes = boxes / old
    if not return_percent_coords:
        new_boxes = new_boxes * torch.tensor([dims[1], dims[0], dims[1], dims[0]], dtype=torch.float32)[None]
    return new_image, new_boxes


def resize_keep(image, boxes, dims, return_percent_coords=True):
    """transforms.py:257-289: as ``resize``, with (H, W) swapped when needed so a landscape image
    stays landscape (and a portrait one portrait)."""
    width, height = image.size
    if width > height:
        if dims[0] < dims[1]:
            dims = (dims[1], dims[0])
    elif dims[0] > dims[1]:
        dims = (dims[1], dims[0])
    return resize(image, boxes, dims, return_percent_coords)


def photometric_distort(image):
    """transforms.py:292-320: brightness, contrast, saturation and hue, shuffled, each applied
    with probability 0.5; factors U(0.5, 1.5), hue U(-18/255, 18/255).  Same draws, same order."""
    new_image = image
    ops = list(DISTORTIONS)
    random.shuffle(ops)
    for d in ops:
        if random.random() < 0.5:
            if d.__name__ == 'adjust_hue':
                f = random.uniform(-18 / 255., 18 / 255.)
            else:
                f = random.uniform(0.5, 1.5)
            new_image = d(new_image, f)
    return new_image


def _cfg(config, key, default=None):
    if isinstance(config, dict):
        return config.get(key, default)
    return getattr(config, key, default)


def transform(image, boxes, labels, split, resize_dim, config):
    """transforms.py:323-383.  TRAIN: photometric distortion, then expand / random_crop (each
    with probability 0.5, when listed in ``config.model['operation_list']``), flip with 0.5.
    Every split: resize (fractional coordinates unless ``return_percent_coords`` is False),
    to_tensor, ImageNet normalisation."""
    assert split in {'TRAIN', 'TEST', 'VAL'}
    model = _cfg(config, 'model', {}) or {}
    ops = model['operation_list']
    percent = model['return_percent_coords']
    new_image, new_boxes, new_labels = image, boxes, labels
    if split == 'TRAIN':
        new_image = to_tensor(photometric_distort(new_image))
        if random.random() < 0.5 and 'expand' in ops:
            new_image, new_boxes = expand(new_image, boxes, filler=IMAGENET_MEAN)
        if random.random() < 0.5 and 'random_crop' in ops:
            new_image, new_boxes, new_labels = random_crop(new_image, new_boxes, new_labels)
        new_image = to_pil(new_image)
        if random.random() < 0.5:
            new_image, new_boxes = flip(new_image, new_boxes)
    new_image, new_boxes = resize(new_image, new_boxes, dims=resize_dim, return_percent_coords=percent)
    return normalize(to_tensor(new_image)), new_boxes, new_labels
