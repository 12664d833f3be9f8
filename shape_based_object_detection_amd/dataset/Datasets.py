"""The reference's on-disk dataset format and its batch format.

On disk (dataset/voc_data_parsing.py:90-95, 121-124): ``{SPLIT}_images.json`` (list of image
paths), ``{SPLIT}_objects.json`` (per image ``{'bbox' | 'boxes': [[x1, y1, x2, y2] in pixels],
'labels': [...], 'difficulties': [...] [, 'image_id']}``) and ``label_map.json`` (name -> id,
background = 0).  In memory: ``collate_fn`` returns ``images [B,3,H,W]`` plus LISTS of per-image
``boxes [G_i,4]`` (fractional xyxy), ``labels [G_i]``, ids and difficulties
(dataset/Datasets.py:58-86) — exactly what the criteria, ``core.pack_gt`` and
``core.GtStaging.stage`` consume.

The readers run on the host in DataLoader workers, as in the reference (dataset/Datasets.py:9-256);
every item goes through ``dataset.transforms.transform`` (transforms.py:323-383, rebuilt at the
same module path with the same random draws).  Images are decoded with PIL.
"""
import json
import os

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

from .transforms import IMAGENET_MEAN, IMAGENET_STD, transform  # noqa: F401  (reference names)

VOC_LABELS = ('aeroplane', 'bicycle', 'bird', 'boat', 'bottle', 'bus', 'car', 'cat', 'chair', 'cow',
              'diningtable', 'dog', 'horse', 'motorbike', 'person', 'pottedplant', 'sheep', 'sofa',
              'train', 'tvmonitor')
VOC_LABEL_MAP = dict({k: v + 1 for v, k in enumerate(VOC_LABELS)}, background=0)   # voc_data_parsing.py:8-9


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


class TrafficDataset(Dataset):
    """dataset/Datasets.py:167-256: several data folders given as ONE space-separated string;
    each folder's ``{split}_images.json`` / ``{split}_objects.json`` are concatenated, folders
    without that split are skipped.  Objects carry ``boxes``, ``labels``, ``difficulties`` and
    ``image_id`` (the item's id)."""

    def __init__(self, data_folder_list, split, input_size, config):
        self.split = split.upper()
        assert self.split in {'TRAIN', 'TEST', 'VAL'}
        self.input_size, self.config = input_size, config
        self.data_folder_list = data_folder_list.split(' ')
        self.images, self.objects = [], []
        for folder in self.data_folder_list:
            path = os.path.join(folder, self.split + '_images.json')
            if not os.path.exists(path):
                continue
            with open(path) as f:
                self.images += json.load(f)
            with open(os.path.join(folder, self.split + '_objects.json')) as f:
                self.objects += json.load(f)
        assert len(self.images) == len(self.objects)

    def __getitem__(self, i):
        image = Image.open(self.images[i], mode='r').convert('RGB')
        obj = self.objects[i]
        boxes = torch.tensor(obj['boxes'], dtype=torch.float32).reshape(-1, 4)
        labels = torch.tensor(obj['labels'], dtype=torch.int64)
        difficulties = torch.tensor(obj['difficulties'], dtype=torch.int64)
        image, boxes, labels = transform(image, boxes, labels, split=self.split,
                                         resize_dim=self.input_size, config=self.config)
        return image, boxes, labels, obj['image_id'], difficulties

    def __len__(self):
        return len(self.images)

    def collate_fn(self, batch):
        """Datasets.py:228-256 (a method here, as in the reference)."""
        return PascalVOCDataset.collate_fn(batch)


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
