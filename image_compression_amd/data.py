"""Host data path, re-designed for the device:
the reference decodes to uint8, converts to fp32 and normalises on the host
(data_utils/transforms/transforms.py ToTensor + ChannelFirst + Normalize), then
copies fp32 batches to the GPU.  Here the loader keeps uint8 HWC crops (1 byte
per channel: a quarter of the PCIe traffic) in pinned memory and
`to_device_input` expands them on the GPU with one kernel
(ic_images_u8_to_input: x/255, (x - mean)/std, HWC -> NCHW).

Semantics mirrored from the reference:
* `KodakDataset(folder)` — sorted glob of the folder, PIL RGB, id = file name
  without ".png" (data_utils/dataset/kodak_dataset.py:25-58); "val" mode has no
  augmentation.
* `ImageNetDataset(folder, metadata_csv)` — the csv's "path" column, id = file
  name without ".jpg" (imagenet_dataset.py:25-60); "train" mode applies
  `RandomCrop(cfg.DATA.SIZE)` with numpy's global RNG exactly like
  transforms.py:129-166 (x then y from np.random.randint; no padding).
* `TrainingSampler(size, shuffle, seed)` — infinite torch.randperm stream with
  a seeded generator (data_utils/sampler.py:24-40); batches with drop_last.
"""
import csv
import ctypes
import glob
import os

import numpy as np
import torch
from PIL import Image

from . import _lib


class RandomCrop:
    """transforms.py:129-166 (numpy global RNG, no padding)."""

    def __init__(self, size):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def __call__(self, image):
        w, h = image.size
        cw, ch = self.size
        if not (w >= cw and h >= ch):
            raise AssertionError(f"got under-sized image {w}x{h} for crop size {cw}x{ch}")
        x = np.random.randint(w - cw + 1)
        y = np.random.randint(h - ch + 1)
        return image.crop((x, y, x + cw, y + ch))


def _to_u8(image):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(image, dtype=np.uint8)))  # H x W x C


class KodakDataset(torch.utils.data.Dataset):
    def __init__(self, data_folder, mode="val", crop=None):
        self.paths = sorted(glob.glob(f"{data_folder}/*"))
        self.crop = RandomCrop(crop) if (mode == "train" and crop) else None

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, idx):
        path = self.paths[idx]
        img = Image.open(path).convert("RGB")
        if self.crop is not None:
            img = self.crop(img)
        return os.path.split(path)[-1].replace(".png", ""), _to_u8(img)


class ImageNetDataset(torch.utils.data.Dataset):
    def __init__(self, data_folder, metadata, mode="train", crop=192):
        self.data_folder = data_folder
        with open(metadata, newline="") as f:
            self.paths = [row["path"] for row in csv.DictReader(f)]
        self.crop = RandomCrop(crop) if (mode == "train" and crop) else None

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, idx):
        path = self.paths[idx]
        img = Image.open(os.path.join(self.data_folder, path)).convert("RGB")
        if self.crop is not None:
            img = self.crop(img)
        return os.path.split(path)[-1].replace(".jpg", ""), _to_u8(img)


class TrainingSampler(torch.utils.data.Sampler):
    """data_utils/sampler.py:24-40."""

    def __init__(self, size, shuffle=True, seed=0):
        self._size, self._shuffle, self._seed = size, shuffle, int(seed)

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self._seed)
        while True:
            if self._shuffle:
                yield from torch.randperm(self._size, generator=g).tolist()
            else:
                yield from range(self._size)


class Batch:
    """data_utils/batch.py: ids + stacked uint8 images [N, H, W, C] (pinned)."""

    def __init__(self, data):
        ids, imgs = zip(*data)
        self.image_ids = ids
        self.imgs = torch.stack(list(imgs))

    def pin_memory(self):
        self.imgs = self.imgs.pin_memory()
        return self


def collate(data):
    return Batch(data)


def infinite_loader(dataset, batch_size, seed=0, num_workers=0):
    """data_utils/dataloader.py:29-57 (train): infinite sampler, drop_last batches."""
    sampler = torch.utils.data.BatchSampler(TrainingSampler(len(dataset), True, seed), batch_size, drop_last=True)
    return torch.utils.data.DataLoader(dataset, batch_sampler=sampler, num_workers=num_workers,
                                       collate_fn=collate, pin_memory=torch.cuda.is_available())


def to_device_input(imgs_u8, device, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0)):
    """uint8 [N, H, W, C] (host or device) -> fp32 [N, C, H, W] model input on
    `device`: (x / 255 - mean) / std on the GPU (transforms.py:88-113)."""
    x = imgs_u8.to(device, non_blocking=True)
    if x.dtype != torch.uint8 or x.dim() != 4:
        raise RuntimeError("to_device_input: uint8 [N, H, W, C] expected")
    if not x.is_cuda:
        raise RuntimeError("imgcomp: HIP kernels need tensors on a ROCm (cuda) device")
    N, H, W, C = x.shape
    sn, sh, sw, sc = x.stride()
    if sc != 1:
        x = x.contiguous()
        sn, sh, sw, sc = x.stride()
    y = torch.empty((N, C, H, W), device=x.device, dtype=torch.float32)
    m = (ctypes.c_float * C)(*[float(v) for v in mean[:C]])
    s = (ctypes.c_float * C)(*[float(v) for v in std[:C]])
    _lib.check(_lib.load().ic_images_u8_to_input(ctypes.c_void_p(x.data_ptr()), sn, sh, sw, N, C, H, W,
                                                 ctypes.cast(m, ctypes.c_void_p), ctypes.cast(s, ctypes.c_void_p),
                                                 _lib.ptr(y), _lib.stream_of(y)), "images_u8_to_input")
    return y
