"""VGG16 (torchvision topology) on the HIP kernels, plus its transfer-learning variant.

Reference parity: ``models.vgg16(pretrained=True)``
(another_neural_net.py:244; printout pytorch_training_inference_on_image.ipynb:1991-2041): 13
conv3x3(pad 1)+bias+ReLU in 5 stages (64,64 | 128,128 | 256x3 | 512x3 | 512x3) each followed by
MaxPool2d(2,2); AdaptiveAvgPool2d(7,7) (the identity at 224x224 input, asserted); classifier
Linear(25088,4096)-ReLU-Dropout(0.5)-Linear(4096,4096)-ReLU-Dropout(0.5)-Linear(4096,1000).
Transfer learning (another_neural_net.py:247-255): backbone frozen, ``classifier[6]`` replaced by
``Linear(4096,256)-ReLU-Dropout(0.4)-Linear(256,10)-LogSoftmax``.

NHWC note: the flatten before the classifier is in (H, W, C) order; ``load_torchvision`` permutes
the first classifier weight from torchvision's (C, H, W) order accordingly.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops import _lib
from ..ops.kernels import K
from .layers import Conv2d, Dropout, Linear, MaxPool2d, MLPHead
from .resnet import STEM_CIN_PAD

CFG16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


class VGG(nn.Module):
    def __init__(self, cfg=CFG16, num_classes=1000, compute_dtype=None):
        super().__init__()
        layers, cin, first = [], 3, True
        for v in cfg:
            if v == "M":
                layers.append(MaxPool2d(2, 2))
            else:
                layers.append(Conv2d(cin, v, 3, 1, 1, bias=True, relu=True, cin_pad=STEM_CIN_PAD if first else None))
                cin, first = v, False
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(
            Linear(512 * 7 * 7, 4096, relu=True), Dropout(0.5),
            Linear(4096, 4096, relu=True), Dropout(0.5),
            Linear(4096, num_classes))
        self.compute_dtype = compute_dtype

    def _cdtype(self, device):
        if self.compute_dtype is not None:
            return self.compute_dtype
        return _lib.default_compute_dtype(device)

    def prepare_input(self, x):
        dt = self._cdtype(x.device)
        if dt == torch.bfloat16:
            scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
            h = K.nchw_to_nhwc(x.contiguous(), STEM_CIN_PAD, scale, None, None)
        else:   # fp32: the reference precision
            scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
            h = K.nchw_to_nhwc_f32(x.contiguous(), STEM_CIN_PAD, scale)
        return h.to(dt)

    def features_flat(self, x):
        h = self.features(self.prepare_input(x))
        assert h.shape[1] == 7 and h.shape[2] == 7, "AdaptiveAvgPool2d(7,7) implemented for 224x224 input only"
        return h.reshape(h.shape[0], -1)

    def forward_logits(self, x):
        f = self.features_flat(x)
        head = self.classifier
        for i, mod in enumerate(head):
            if i == len(head) - 1 and hasattr(mod, "forward_logits"):
                return mod.forward_logits(f)
            f = mod(f)
        return f

    def forward(self, x):
        return self.classifier(self.features_flat(x))

    def freeze_backbone(self):
        """another_neural_net.py:247-248 (all params frozen before the head is replaced)."""
        for p in self.parameters():
            p.requires_grad_(False)
        return self

    def replace_head(self, head: nn.Module):
        self.classifier[-1] = head
        return self

    @torch.no_grad()
    def load_torchvision(self, sd: dict, load_head: bool | None = None):
        convs = [m for m in self.features if isinstance(m, Conv2d)]
        keys = sorted({k.rsplit(".", 1)[0] for k in sd if k.startswith("features.")}, key=lambda s: int(s.split(".")[1]))
        for conv, k in zip(convs, keys):
            w = sd[k + ".weight"]
            conv.weight.zero_()
            conv.weight[..., : w.shape[1]].copy_(w.permute(0, 2, 3, 1))
            conv.bias.copy_(sd[k + ".bias"])
        w0 = sd["classifier.0.weight"].view(4096, 512, 7, 7).permute(0, 2, 3, 1).reshape(4096, -1)
        self.classifier[0].load_torch(w0, sd["classifier.0.bias"])
        self.classifier[2].load_torch(sd["classifier.3.weight"], sd["classifier.3.bias"])
        w6 = sd.get("classifier.6.weight")
        head = self.classifier[-1]
        if load_head is not False and isinstance(head, Linear) and w6 is not None and \
                tuple(w6.shape) == (head.out_features, head.in_features):
            head.load_torch(w6, sd["classifier.6.bias"])
        elif load_head:
            raise ValueError("load_torchvision: head weights missing or of another shape")
        for p in self.parameters():   # bf16 compute shadows of a flat arena follow the new masters
            owner = getattr(p, "_flat_owner", None)
            if owner is not None:
                owner.refresh_shadows()
                break
        return self


def vgg16(num_classes=1000, **kw):
    return VGG(CFG16, num_classes, **kw)


def vgg16_transfer(num_classes=10, hidden=256, p=0.4, **kw):
    """The reference's VGG16 TL model (another_neural_net.py:244-255)."""
    m = vgg16(1000, **kw).freeze_backbone()
    return m.replace_head(MLPHead(4096, hidden, num_classes, p))
