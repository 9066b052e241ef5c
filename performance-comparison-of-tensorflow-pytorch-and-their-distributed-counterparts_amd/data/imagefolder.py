"""Real-folder image pipeline (optional) — PIL decode on a thread pool.

Parity with the reference's torchvision usage:
  * ``ImageFolder`` — ``root/<class>/*`` sorted classes, (path, class_index) samples;
  * ``load_split_train_test`` — B1/B2: ``Resize((224,224)) + ToTensor`` (no Normalize), shuffle
    indices, 80/20 split, batch 64, either ``SubsetRandomSampler`` semantics (notebook) or the
    distributed variant with :class:`ShardedSampler` (``reference_index_bug`` reproduces the
    script's list-of-indices bug on request);
  * ``get_random_images`` — B3, one batch of ``num`` random images (+ labels);
  * ``get_image_paths`` — B4, walks ``root/<class>/*.JPEG`` and prints the count;
  * ``train_augment`` / ``valid_transform`` — B5 (RandomResizedCrop(256,(0.8,1)), rotation 15,
    flip, CenterCrop 224, ToTensor, ImageNet Normalize) / (Resize 256, CenterCrop 224, ...);
  * ``preprocess_single`` — B6; Keras variants in :mod:`pcmp.models.keras_resnet` (B7/B8).
Decoded batches are uint8 NCHW host tensors (pinned when a GPU is present); the fused device
kernel ``nchw_to_nhwc`` does the /255 scaling and layout change on the GPU.  With
``device_resize=True`` (the default when batches go to a GPU) the host only decodes the JPEG: the
raw uint8 HWC image is copied to the device and ``resize_image`` (csrc/elementwise.hip) runs
Pillow's bilinear resize there, bit-identical to ``PIL.Image.resize(..., BILINEAR)``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import random

import numpy as np
import torch

from ..parallel.sampler import ShardedSampler

IMG_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".JPEG", ".JPG", ".PNG")
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _pil():
    from PIL import Image
    return Image


class ImageFolder:
    def __init__(self, root, size=224):
        self.root = root
        self.classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.samples = []
        for c in self.classes:
            for f in sorted(os.listdir(os.path.join(root, c))):
                if f.endswith(IMG_EXT):
                    self.samples.append((os.path.join(root, c, f), self.class_to_idx[c]))
        self.size = size
        self.pool = cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4))

    def __len__(self):
        return len(self.samples)

    def load(self, i):
        """Resize((224,224)) + ToTensor-equivalent as uint8 CHW (scaling happens on device)."""
        Image = _pil()
        path, y = self.samples[i]
        with Image.open(path) as im:
            im = im.convert("RGB").resize((self.size, self.size), Image.BILINEAR)
            a = np.asarray(im, dtype=np.uint8)
        return torch.from_numpy(a.copy()).permute(2, 0, 1), y

    def load_raw(self, i):
        """Decode only: uint8 HWC at the file's own size (the resize runs on the device)."""
        Image = _pil()
        path, y = self.samples[i]
        with Image.open(path) as im:
            a = np.asarray(im.convert("RGB"), dtype=np.uint8)
        return torch.from_numpy(a.copy()), y

    def get_batch(self, idx, device=None, device_resize=None):
        on_gpu = device is not None and torch.device(device).type == "cuda"
        if device_resize is None:
            device_resize = on_gpu
        if device_resize and on_gpu:
            items = list(self.pool.map(self.load_raw, list(idx)))
            x = torch.cat([resize_on_device(t, self.size, device) for t, _ in items])
            y = torch.tensor([l for _, l in items], dtype=torch.long).to(device, non_blocking=True)
            return x, y
        items = list(self.pool.map(self.load, list(idx)))
        x = torch.stack([t for t, _ in items])
        y = torch.tensor([l for _, l in items], dtype=torch.long)
        if on_gpu:
            x = x.pin_memory().to(device, non_blocking=True)
            y = y.to(device, non_blocking=True)
        return x, y


def resize_on_device(img_hwc_u8: torch.Tensor, size, device, out="u8", cpad=8, scale=1.0, mean=None, std=None):
    """One decoded image (uint8 HWC, host) -> device, Pillow-exact bilinear resize to ``size`` there.
    ``out="u8"``: uint8 [1,3,S,S] (ToTensor happens in the model's input conversion); ``"bf16"`` /
    ``"f32"``: the fused model input, NHWC [1,S,S,cpad] of (u8 * scale - mean) / std."""
    from ..ops.kernels import K
    s = (size, size) if isinstance(size, int) else tuple(size)
    x = img_hwc_u8
    if x.dim() == 3:
        x = x.unsqueeze(0)
    if not x.is_cuda:
        x = x.pin_memory().to(device, non_blocking=True)
    mode = {"u8": 0, "bf16": 1, "f32": 2}[out]
    if mean is not None:
        mean = torch.as_tensor(mean, dtype=torch.float32, device=x.device)
        std = torch.as_tensor(std, dtype=torch.float32, device=x.device)
    return K.resize_image(x.contiguous(), s[0], s[1], mode, cpad, scale, mean, std)


def load_split_train_test(datadir, valid_size=0.2, batch_size=64, distributed=False, device=None,
                          reference_index_bug=False, seed=None):
    from .synthetic import BatchLoader
    data = ImageFolder(datadir)
    n = len(data)
    indices = list(range(n))
    split = int(np.floor(valid_size * n))
    rng = np.random.RandomState(seed) if seed is not None else np.random
    rng.shuffle(indices)
    train_idx, test_idx = indices[split:], indices[:split]
    if distributed:
        tr = BatchLoader(data, batch_size, ShardedSampler(train_idx, reference_index_bug=reference_index_bug), device)
        te = BatchLoader(data, batch_size, ShardedSampler(test_idx, reference_index_bug=reference_index_bug), device)
    else:
        tr = BatchLoader(data, batch_size, device=device, indices=train_idx, shuffle=True)
        te = BatchLoader(data, batch_size, device=device, indices=test_idx, shuffle=True)
    print(data.classes)
    return tr, te


def flow_from_directory(directory, target_size=224, batch_size=64, device=None, distributed=False, seed=0):
    """B8: Keras ``ImageDataGenerator(rescale=1./255).flow_from_directory(directory,
    target_size=(224,224), batch_size=64, class_mode="categorical", shuffle=True)`` (resnet.py:10-16).
    Batches are uint8 NCHW (the model's input conversion applies the 1/255 rescale on the device)
    with integer labels; ``keras_fit`` one-hot encodes them (categorical).  Prints Keras' "Found N
    images belonging to K classes." line."""
    from .synthetic import BatchLoader
    data = ImageFolder(directory, size=target_size)
    print(f"Found {len(data)} images belonging to {len(data.classes)} classes.")
    if distributed:
        return BatchLoader(data, batch_size, ShardedSampler(len(data), shuffle=True, seed=seed), device)
    return BatchLoader(data, batch_size, device=device, shuffle=True, seed=seed)


def get_random_images(dataset, num, distributed=False, device=None):
    indices = list(range(len(dataset)))
    random.shuffle(indices)
    idx = indices[:num]
    if distributed:
        idx = list(iter(ShardedSampler(idx)))
    return dataset.get_batch(idx, device)


def get_image_paths(root):
    """another_neural_net.py:18-35 / Standalone_Inference_Imagenette_trial.ipynb:74-91 (no chdir)."""
    paths = []
    for d in sorted(os.listdir(root)):
        paths += sorted(glob.glob(os.path.join(root, d, "*.JPEG")))
    print(len(paths))
    return paths


def preprocess_single(path, size=224, device=None):
    """B6: PIL open -> RGB -> Resize -> ToTensor -> unsqueeze(0) (float NCHW in [0,1]).  With a GPU
    ``device`` only the decode runs on the host; the resize runs on the device (``resize_image``)."""
    Image = _pil()
    with Image.open(path) as im:
        im = im.convert("RGB")
        if device is not None and torch.device(device).type == "cuda":
            raw = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy())
            return resize_on_device(raw, size, device).float() / 255.0
        a = np.asarray(im.resize((size, size), Image.BILINEAR), dtype=np.float32) / 255.0
    return torch.from_numpy(a).permute(2, 0, 1).unsqueeze(0)


def valid_transform(img, size=224):
    """B5 'valid': Resize(256) -> CenterCrop(224) -> ToTensor -> Normalize (ImageNet)."""
    Image = _pil()
    w, h = img.size
    s = 256 / min(w, h)
    img = img.resize((max(1, round(w * s)), max(1, round(h * s))), Image.BILINEAR)
    w, h = img.size
    l, t = (w - size) // 2, (h - size) // 2
    img = img.crop((l, t, l + size, t + size))
    a = (np.asarray(img, dtype=np.float32) / 255.0 - IMAGENET_MEAN) / IMAGENET_STD
    return torch.from_numpy(a.astype(np.float32)).permute(2, 0, 1)


def train_augment(img, size=224, rng=random):
    """B5 'train': RandomResizedCrop(256,(0.8,1)) -> RandomRotation(15) -> ColorJitter() (identity
    at default args) -> RandomHorizontalFlip -> CenterCrop(224) -> ToTensor -> Normalize."""
    Image = _pil()
    w, h = img.size
    area = w * h * rng.uniform(0.8, 1.0)
    ratio = np.exp(rng.uniform(np.log(3 / 4), np.log(4 / 3)))
    cw = int(round(np.sqrt(area * ratio)))
    ch = int(round(np.sqrt(area / ratio)))
    cw, ch = min(cw, w), min(ch, h)
    l, t = rng.randint(0, w - cw), rng.randint(0, h - ch)
    img = img.crop((l, t, l + cw, t + ch)).resize((256, 256), Image.BILINEAR)
    img = img.rotate(rng.uniform(-15, 15))
    if rng.random() < 0.5:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
    o = (256 - size) // 2
    img = img.crop((o, o, o + size, o + size))
    a = (np.asarray(img, dtype=np.float32) / 255.0 - IMAGENET_MEAN) / IMAGENET_STD
    return torch.from_numpy(a.astype(np.float32)).permute(2, 0, 1)


IMAGENETTE_LABELS = {  # Standalone_Inference_Imagenette_trial.ipynb:161-162 (label_names)
    0: "tench", 1: "English springer", 2: "cassette player", 3: "chain saw", 4: "church",
    5: "French horn", 6: "garbage truck", 7: "gas pump", 8: "golf ball", 9: "parachute",
}
