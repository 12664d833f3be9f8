"""The reference's on-disk dataset format and its batch format.

On disk (dataset/voc_data_parsing.py:90-95, 121-124): ``{SPLIT}_images.json`` (list of image
paths), ``{SPLIT}_objects.json`` (per image ``{'bbox' | 'boxes': [[x1, y1, x2, y2] in pixels],
'labels': [...], 'difficulties': [...] [, 'image_id']}``) and ``label_map.json`` (name -> id,
background = 0).  In memory: ``collate_fn`` returns ``images [B,3,H,W]`` plus LISTS of per-image
``boxes [G_i,4]`` (fractional xyxy), ``labels [G_i]``, ids and difficulties
(dataset/Datasets.py:58-86) — exactly what the criteria, ``core.pack_gt`` and
``core.GtStaging.stage`` consume.

The readers and the geometric transforms that touch boxes (resize to fractional coordinates,
flip, expand, random_crop with its IoU test) run on the host in DataLoader workers, as in the
reference (dataset/Datasets.py:9-86, dataset/transforms.py:86-254, 323-383); random_crop's IoU is
``metrics.find_jaccard_overlap`` on CPU tensors, i.e. the drop-in's host path.  Pixel-only
photometric distortion (transforms.py:292-320) is not rebuilt: it never touches boxes and needs
torchvision's colour ops, which this image lacks.  Images are decoded with PIL; resizing uses
PIL's bilinear filter (what torchvision's functional resize does for PIL images).
"""
import json
import os
import random

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

from .. import metrics

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # transforms.py:341-342
IMAGENET_STD = (0.229, 0.224, 0.225)

VOC_LABELS = ('aeroplane', 'bicycle', 'bird', 'boat', 'bottle', 'bus', 'car', 'cat', 'chair', 'cow',
              'diningtable', 'dog', 'horse', 'motorbike', 'person', 'pottedplant', 'sheep', 'sofa',
              'train', 'tvmonitor')
VOC_LABEL_MAP = dict({k: v + 1 for v, k in enumerate(VOC_LABELS)}, background=0)   # voc_data_parsing.py:8-9


def _cfg(config, key, default=None):
    if isinstance(config, dict):
        return config.get(key, default)
    return getattr(config, key, default)


# ----------------------------------------------------------------------------- transforms
def to_tensor(image):
    """PIL RGB -> float [3,H,W] in [0,1]."""
    a = np.asarray(image, dtype=np.uint8)
    return torch.from_numpy(a.astype(np.float32) / 255.0).permute(2, 0, 1).contiguous()


def to_pil(t):
    a = (t.clamp(0, 1) * 255.0).round().to(torch.uint8).permute(1, 2, 0).numpy()
    return Image.fromarray(a, mode='RGB')


def normalize(t, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    m = torch.tensor(mean, dtype=t.dtype).view(3, 1, 1)
    s = torch.tensor(std, dtype=t.dtype).view(3, 1, 1)
    return (t - m) / s


def resize(image, boxes, dims, return_percent_coords=True):
    """transforms.py:230-254: PIL resize to dims = (H, W); boxes / (w, h, w, h) (fractional), or
    rescaled to the new pixel size."""
    new_image = image.resize((dims[1], dims[0]), Image.BILINEAR)
    old = torch.tensor([image.width, image.height, image.width, image.height], dtype=torch.float32)[None]
    new_boxes = boxes / old
    if not return_percent_coords:
        new_boxes = new_boxes * torch.tensor([dims[1], dims[0], dims[1], dims[0]], dtype=torch.float32)[None]
    return new_image, new_boxes


def flip(image, boxes):
    """transforms.py:210-227: horizontal flip of the image and the pixel boxes."""
    new_image = image.transpose(Image.FLIP_LEFT_RIGHT)
    new_boxes = boxes.clone()
    new_boxes[:, 0] = image.width - boxes[:, 0] - 1
    new_boxes[:, 2] = image.width - boxes[:, 2] - 1
    return new_image, new_boxes[:, [2, 1, 0, 3]]


def expand(image, boxes, filler, rng=random):
    """transforms.py:86-122: place the [3,H,W] image on a canvas up to 4x larger filled with
    `filler` (zoom out); pixel boxes shifted by the placement."""
    h, w = image.shape[1:]
    scale = rng.uniform(1, 4)
    nh, nw = int(scale * h), int(scale * w)
    new_image = torch.tensor(filler, dtype=torch.float32).view(3, 1, 1).expand(3, nh, nw).clone()
    left, top = rng.randint(0, nw - w), rng.randint(0, nh - h)
    new_image[:, top:top + h, left:left + w] = image
    return new_image, boxes + torch.tensor([left, top, left, top], dtype=torch.float32)[None]


def random_crop(image, boxes, labels, rng=random, max_trials=50):
    """transforms.py:125-207: random crop [3,H,W] with a minimum-overlap requirement drawn from
    {0, .1, .3, .5, .7, .9, None}; the IoU test is find_jaccard_overlap on CPU tensors (the host
    path).  Keeps objects whose centres fall inside the crop, clipped to it."""
    h, w = image.shape[1:]
    while True:
        min_overlap = rng.choice([0., .1, .3, .5, .7, .9, None])
        if min_overlap is None:
            return image, boxes, labels
        for _ in range(max_trials):
            nh, nw = int(rng.uniform(0.3, 1) * h), int(rng.uniform(0.3, 1) * w)
            if not 0.5 < nh / nw < 2:
                continue
            left, top = rng.randint(0, w - nw), rng.randint(0, h - nh)
            crop = torch.tensor([left, top, left + nw, top + nh], dtype=torch.float32)
            overlap = metrics.find_jaccard_overlap(crop[None], boxes).squeeze(0)
            if overlap.max().item() < min_overlap:
                continue
            centers = (boxes[:, :2] + boxes[:, 2:]) / 2.
            inside = ((centers[:, 0] > left) & (centers[:, 0] < crop[2]) &
                      (centers[:, 1] > top) & (centers[:, 1] < crop[3]))
            if not inside.any():
                continue
            nb = boxes[inside].clone()
            nb[:, :2] = torch.max(nb[:, :2], crop[:2]) - crop[:2]
            nb[:, 2:] = torch.min(nb[:, 2:], crop[2:]) - crop[:2]
            return image[:, top:top + nh, left:left + nw], nb, labels[inside]


def transform(image, boxes, labels, split, resize_dim, config, rng=random):
    """transforms.py:323-383 without the pixel-only photometric step: TRAIN = expand / crop when
    listed in ``config.model['operation_list']`` (each with probability 0.5), flip with 0.5;
    every split = resize (fractional coordinates unless ``return_percent_coords`` is False),
    to_tensor, ImageNet normalisation."""
    split = split.upper()
    assert split in {'TRAIN', 'TEST', 'VAL'}
    model = _cfg(config, 'model', {}) or {}
    ops = model.get('operation_list', []) or []
    percent = model.get('return_percent_coords', True)
    new_image, new_boxes, new_labels = image, boxes, labels
    if split == 'TRAIN':
        t = to_tensor(new_image)
        if rng.random() < 0.5 and 'expand' in ops:
            t, new_boxes = expand(t, new_boxes, IMAGENET_MEAN, rng)
        if rng.random() < 0.5 and 'random_crop' in ops:
            t, new_boxes, new_labels = random_crop(t, new_boxes, new_labels, rng)
        new_image = to_pil(t)
        if rng.random() < 0.5:
            new_image, new_boxes = flip(new_image, new_boxes)
    new_image, new_boxes = resize(new_image, new_boxes, resize_dim, percent)
    return normalize(to_tensor(new_image)), new_boxes, new_labels


# ----------------------------------------------------------------------------- datasets
class PascalVOCDataset(Dataset):
    """dataset/Datasets.py:9-86: ``{split}_images.json`` / ``{split}_objects.json`` in
    ``data_folder``; items (image [3,H,W], boxes [G,4], labels [G], image path, difficulties)."""

    def __init__(self, data_folder, split, input_size, config):
        self.split = split.upper()
        assert self.split in {'TRAIN', 'TEST', 'VAL'}
        assert config is not None
        self.input_size, self.config, self.data_folder = input_size, config, data_folder
        with open(os.path.join(data_folder, self.split + '_images.json')) as f:
            self.images = json.load(f)
        with open(os.path.join(data_folder, self.split + '_objects.json')) as f:
            self.objects = json.load(f)
        assert len(self.images) == len(self.objects)

    def _id(self, i):
        return self.images[i]

    def __getitem__(self, i):
        image = Image.open(self.images[i], mode='r').convert('RGB')
        obj = self.objects[i]
        boxes = torch.tensor(obj['bbox'] if 'bbox' in obj else obj['boxes'], dtype=torch.float32).reshape(-1, 4)
        labels = torch.tensor(obj['labels'], dtype=torch.int64)
        difficulties = torch.tensor(obj['difficulties'], dtype=torch.int64)
        image, boxes, labels = transform(image, boxes, labels, split=self.split,
                                         resize_dim=self.input_size, config=self.config)
        return image, boxes, labels, self._id(i), difficulties

    def __len__(self):
        return len(self.images)

    @staticmethod
    def collate_fn(batch):
        """Datasets.py:58-86: stacked images, LISTS of per-image boxes / labels / ids /
        difficulties (each image has its own number of objects)."""
        images, boxes, labels, ids, diffs = [], [], [], [], []
        for b in batch:
            images.append(b[0])
            boxes.append(b[1])
            labels.append(b[2])
            ids.append(b[3])
            diffs.append(b[4])
        return torch.stack(images, dim=0), boxes, labels, ids, diffs


class COCO17Dataset(PascalVOCDataset):
    """dataset/Datasets.py:89-164: same files, the id is the object record's ``image_id``."""

    def _id(self, i):
        return self.objects[i]['image_id']


def read_label_map(data_folder):
    """``label_map.json`` (voc_data_parsing.py:94-95): class name -> id, background 0."""
    with open(os.path.join(data_folder, 'label_map.json')) as f:
        return json.load(f)


def write_synthetic_voc(folder, n_images, size=(300, 300), split='TRAIN', seed=0, max_objects=8):
    """A VOC-format data folder of ``n_images`` synthetic JPEGs (BASELINE config C1's '4 synthetic
    VOC-format images'): random noise images, random pixel boxes (1..max_objects per image,
    VOC's 0-based integer corners), labels 1..20, no difficult objects."""
    os.makedirs(folder, exist_ok=True)
    rng = np.random.RandomState(seed)
    images, objects = [], []
    h, w = size
    for i in range(n_images):
        path = os.path.join(folder, '%06d.jpg' % i)
        Image.fromarray(rng.randint(0, 256, (h, w, 3), dtype=np.uint8), mode='RGB').save(path, quality=90)
        g = int(rng.randint(1, max_objects + 1))
        x1 = rng.randint(0, w - 20, g)
        y1 = rng.randint(0, h - 20, g)
        x2 = np.minimum(x1 + rng.randint(10, w // 2, g), w - 1)
        y2 = np.minimum(y1 + rng.randint(10, h // 2, g), h - 1)
        objects.append({'bbox': np.stack([x1, y1, x2, y2], 1).tolist(),
                        'labels': rng.randint(1, 21, g).tolist(), 'difficulties': [0] * g})
        images.append(path)
    with open(os.path.join(folder, split + '_images.json'), 'w') as f:
        json.dump(images, f)
    with open(os.path.join(folder, split + '_objects.json'), 'w') as f:
        json.dump(objects, f)
    with open(os.path.join(folder, 'label_map.json'), 'w') as f:
        json.dump(VOC_LABEL_MAP, f)
    return folder
