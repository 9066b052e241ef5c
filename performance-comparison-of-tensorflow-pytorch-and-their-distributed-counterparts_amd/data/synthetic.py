"""On-device synthetic datasets with the reference's shapes.

No network in this environment: Imagenette2 and the IMDB CSV (its zip is a missing blob,
.MISSING_LARGE_BLOBS:1) are replaced by deterministic synthetic data of the same shapes:
  * ``SyntheticImages``: ``[3, 224, 224]`` float images in [0,1] (what ``ToTensor`` yields),
    10 classes (Imagenette), default size 9,469 (the train split the 119x64 steps imply,
    SURVEY §2.3); class-dependent low-frequency patterns + noise so transfer learning has
    something to learn;
  * ``SyntheticIMDB``: int64 token ids ``[128]`` (vocab 30522, [CLS]=101 ... [SEP]=102, post
    padding 0), a review-length distribution, 2 classes with class-dependent token statistics.
Labels, lengths and class signatures are pure functions of (seed, index), so any sharding or
shuffling sees the same labelled dataset on every rank; the additive noise is drawn per batch.  Batches are generated directly on the target device (no host->device copy); on the GPU
one fused kernel (synth_images) writes the batch.
"""
from __future__ import annotations

import math

import torch


def _hash01(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """Deterministic per-element uniform in [0,1): a 32-bit integer mix (xorshift-multiply) of
    (seed, index), exact in int64 arithmetic on any device."""
    m = 0xFFFFFFFF
    x = (idx.to(torch.int64) * 2654435761 + ((seed * 40503 + 12345) & m)) & m
    for _ in range(2):
        x = x ^ (x >> 16)
        x = (x * 0x45D9F3B) & m
    x = x ^ (x >> 16)
    return (x.double() / 4294967296.0).float()


class SyntheticImages:
    def __init__(self, n=9469, num_classes=10, image_size=224, seed=0, device="cpu", channels=3, noise=0.15):
        self.n, self.num_classes, self.size, self.seed = n, num_classes, image_size, seed
        self.device = torch.device(device)
        self.channels, self.noise = channels, noise
        g = torch.Generator().manual_seed(seed + 1)
        # per-class colour + spatial frequency signature
        self.color = torch.rand(num_classes, channels, 1, 1, generator=g)
        self.freq = 1.0 + 4.0 * torch.rand(num_classes, 2, generator=g)
        self.classes = [f"class_{i}" for i in range(num_classes)]

    def __len__(self):
        return self.n

    def labels(self, idx: torch.Tensor) -> torch.Tensor:
        return (torch.floor(_hash01(self.seed + 7, idx.cpu()) * self.num_classes).long() % self.num_classes)

    def _native_ok(self, dev) -> bool:
        import os

        from ..ops import _lib
        return (dev.type == "cuda" and self.size % 4 == 0 and os.environ.get("PCMP_SYNTH_NATIVE", "1") != "0"
                and _lib.use_native(torch.empty(0, device=dev)))

    def get_batch(self, idx, device=None):
        dev = torch.device(device) if device is not None else self.device
        idx = torch.as_tensor(idx, dtype=torch.long)
        y = self.labels(idx)
        B, S, C = idx.numel(), self.size, self.channels
        seed = int(self.seed * 1000003 + int(idx[0]) * 7919 + B) % (2 ** 62)
        if self._native_ok(dev):
            # one fused launch (csrc/elementwise.hip synth_images_kernel): same formula, counter-based noise
            from ..ops.kernels import K
            if getattr(self, "_dev_tabs", (None,))[0] != dev:
                self._dev_tabs = (dev, self.color.view(self.num_classes, C).contiguous().to(dev),
                                  self.freq.contiguous().to(dev))
            yd = y.to(dev, non_blocking=True)
            return K.synth_images(yd, self._dev_tabs[1], self._dev_tabs[2], S, seed, float(self.noise)), yd
        lin = torch.linspace(0, 2 * math.pi, S, device=dev)
        fy, fx = self.freq[y, 0].to(dev), self.freq[y, 1].to(dev)
        pat = torch.sin(fy.view(B, 1, 1) * lin.view(1, S, 1)) * torch.cos(fx.view(B, 1, 1) * lin.view(1, 1, S))
        g = torch.Generator(device=dev).manual_seed(seed)
        noise = torch.rand(B, C, S, S, device=dev, generator=g)
        x = 0.5 * self.color[y].to(dev) + 0.25 * (pat.unsqueeze(1) + 1.0) * 0.5 + self.noise * noise
        return x.clamp_(0.0, 1.0), y.to(dev)


class SyntheticIMDB:
    VOCAB, CLS, SEP, PAD = 30522, 101, 102, 0

    def __init__(self, n=12500, max_len=128, seed=0, device="cpu", num_classes=2):
        self.n, self.max_len, self.seed = n, max_len, seed
        self.device = torch.device(device)
        self.num_classes = num_classes

    def __len__(self):
        return self.n

    def labels(self, idx):
        return (_hash01(self.seed + 3, torch.as_tensor(idx).cpu()) * self.num_classes).long() % self.num_classes

    def lengths(self, idx):
        # IMDB reviews are long: most are truncated at 128; ~25% shorter (min 8 tokens)
        u = _hash01(self.seed + 11, torch.as_tensor(idx).cpu())
        L = torch.where(u < 0.75, torch.full_like(u, self.max_len), 8 + (u - 0.75) / 0.25 * (self.max_len - 8))
        return L.long().clamp(8, self.max_len)

    def get_batch(self, idx, device=None):
        dev = torch.device(device) if device is not None else self.device
        idx = torch.as_tensor(idx, dtype=torch.long)
        B, S = idx.numel(), self.max_len
        y = self.labels(idx)
        L = self.lengths(idx)
        g = torch.Generator().manual_seed(int(self.seed * 1000003 + int(idx.sum()) * 31 + B) % (2 ** 62))
        tok = torch.randint(1000, self.VOCAB, (B, S), generator=g)
        # class-dependent "sentiment" tokens at random positions
        sent = torch.randint(0, 50, (B, S), generator=g) + 2000 + 500 * y.view(B, 1)
        use = torch.rand(B, S, generator=g) < 0.3
        tok = torch.where(use, sent, tok)
        pos = torch.arange(S).view(1, S)
        tok[:, 0] = self.CLS
        tok = torch.where(pos == (L.view(B, 1) - 1), torch.full_like(tok, self.SEP), tok)
        tok = torch.where(pos >= L.view(B, 1), torch.zeros_like(tok), tok)
        mask = (tok > 0).long()
        return tok.to(dev), mask.to(dev), y.to(dev)


class BatchLoader:
    """Batches over a sampler's index stream; ``get_batch`` generates/loads them on ``device``.
    ``len()`` = number of batches (DataLoader semantics, drop_last=False)."""

    def __init__(self, dataset, batch_size, sampler=None, device=None, indices=None, shuffle=False, seed=0):
        self.ds, self.bs, self.sampler, self.device = dataset, batch_size, sampler, device
        self.indices = indices
        self.shuffle, self.seed, self.epoch = shuffle, seed, 0

    def _index_stream(self):
        if self.sampler is not None:
            return list(iter(self.sampler))
        idx = list(self.indices) if self.indices is not None else list(range(len(self.ds)))
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            perm = torch.randperm(len(idx), generator=g).tolist()
            idx = [idx[i] for i in perm]
        return idx

    def set_epoch(self, e):
        self.epoch = e
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(e)

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else (len(self.indices) if self.indices is not None else len(self.ds))
        return (n + self.bs - 1) // self.bs

    def __iter__(self):
        idx = self._index_stream()
        for i in range(0, len(idx), self.bs):
            yield self.ds.get_batch(idx[i:i + self.bs], self.device)
