"""ResNet-18/34/50/101/152 (torchvision v1.5 topology; Keras v1 variant) on the fused HIP blocks.

Reference parity:
  * ``models.resnet50(pretrained=True)`` of another_neural_net.py:95 /
    pytorch_training_inference_on_image.ipynb:389 — 16 Bottlenecks (3/4/6/3), stride on the 3x3,
    architecture printout at nb :454-635; 25,557,032 params with the 1000-way fc.
  * transfer-learning mode: ``freeze_backbone()`` sets requires_grad=False on every
    backbone parameter while BatchNorm stays in train mode (running stats keep updating, batch
    statistics are used — the reference's behaviour), and ``replace_head(MLPHead(...))`` swaps
    ``fc`` (another_neural_net.py:105-112).
  * ``variant="keras"`` puts the stride on the first 1x1 conv of each downsampling bottleneck
    (Keras ResNet50 v1, resnet.py:17).  Keras' conv biases are omitted: in front of
    a train-mode BatchNorm a per-channel bias is cancelled exactly by the mean subtraction (its
    gradient is identically zero), so they change neither outputs nor training.
  * ResNet-18 (BasicBlock) is the north-star minimum slice.

Input: NCHW float images (as produced by ``ToTensor``) or NHWC bf16 already padded to 8 channels;
``prepare_input`` runs the fused NCHW->NHWC/bf16/pad kernel.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops import _lib
from ..ops.conv_blocks import ResidualBlockFn, StemFn, stem_s2d_wanted
from ..ops.kernels import K
from .layers import Conv2d, ConvBN, GlobalAvgPool, Linear, MLPHead

STEM_CIN_PAD = 8


class Stem(nn.Module):
    def __init__(self, cin=3):
        super().__init__()
        self.conv = ConvBN(cin, 64, 7, stride=2, pad=3, cin_pad=STEM_CIN_PAD)

    def param_list(self):
        return self.conv.params()

    def forward(self, x):
        return StemFn.apply(x, self, *self.param_list())


class _Block(nn.Module):
    def param_list(self):
        ps = []
        for L in self.main_layers():
            ps += L.params()
        if self.down_layer() is not None:
            ps += self.down_layer().params()
        return ps

    def down_layer(self):
        return self.downsample

    def forward(self, x):
        return ResidualBlockFn.apply(x, self, *self.param_list())


class BasicBlock(_Block):
    expansion = 1

    def __init__(self, cin, planes, stride=1, zero_init_residual=False, stride_in_1x1=False):
        super().__init__()
        self.conv1 = ConvBN(cin, planes, 3, stride, 1)
        self.conv2 = ConvBN(planes, planes, 3, 1, 1, zero_init_gamma=zero_init_residual)
        self.downsample = ConvBN(cin, planes, 1, stride, 0) if (stride != 1 or cin != planes) else None

    def main_layers(self):
        return [self.conv1, self.conv2]


class Bottleneck(_Block):
    expansion = 4

    def __init__(self, cin, planes, stride=1, zero_init_residual=False, stride_in_1x1=False):
        super().__init__()
        out = planes * 4
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = ConvBN(cin, planes, 1, s1, 0)
        self.conv2 = ConvBN(planes, planes, 3, s3, 1)
        self.conv3 = ConvBN(planes, out, 1, 1, 0, zero_init_gamma=zero_init_residual)
        self.downsample = ConvBN(cin, out, 1, stride, 0) if (stride != 1 or cin != out) else None

    def main_layers(self):
        return [self.conv1, self.conv2, self.conv3]


_CFG = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
    "resnet101": (Bottleneck, [3, 4, 23, 3]),
    "resnet152": (Bottleneck, [3, 8, 36, 3]),
}


class ResNet(nn.Module):
    def __init__(self, arch="resnet50", num_classes=1000, variant="torchvision", zero_init_residual=False,
                 compute_dtype=None):
        super().__init__()
        block, layers = _CFG[arch]
        self.arch = arch
        self.stem = Stem()
        stride_in_1x1 = variant == "keras"
        cin = 64
        stages = []
        for i, (planes, n) in enumerate(zip([64, 128, 256, 512], layers)):
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(block(cin, planes, stride, zero_init_residual, stride_in_1x1))
                cin = planes * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.avgpool = GlobalAvgPool()
        self.feature_dim = cin
        self.fc = Linear(cin, num_classes)
        self.compute_dtype = compute_dtype

    # ---- dtype / input ---------------------------------------------------------------------
    def _cdtype(self, device):
        if self.compute_dtype is not None:
            return self.compute_dtype
        return _lib.default_compute_dtype(device)

    def prepare_input(self, x):
        """NCHW float/uint8 images -> NHWC compute-dtype, channels padded to 8 (on the GPU: the
        16-channel space-to-depth image the stem convolves, see ops/conv_blocks.py)."""
        dt = self._cdtype(x.device)
        if x.dim() == 4 and x.shape[-1] == STEM_CIN_PAD and x.shape[1] != STEM_CIN_PAD:
            h = x
        elif dt == torch.bfloat16:
            scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
            if x.shape[1] <= 4 and stem_s2d_wanted(x.device):
                # straight to the space-to-depth layout of the GPU stem (ops/conv_blocks.py)
                h = K.image_to_s2d(x.contiguous(), self.stem.conv.pad, scale, None, None, False)
            else:
                h = K.nchw_to_nhwc(x.contiguous(), STEM_CIN_PAD, scale, None, None)
        else:  # fp32 (the reference precision; CPU and --dtype fp32 on the GPU): no bf16 rounding
            scale = 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0
            if x.shape[1] <= 4 and stem_s2d_wanted(x.device):
                h = K.image_to_s2d_f32(x.contiguous(), self.stem.conv.pad, scale)   # fp32 s2d stem image
            else:
                h = K.nchw_to_nhwc_f32(x.contiguous(), STEM_CIN_PAD, scale)
        return h if h.dtype == dt else h.to(dt)

    # ---- forward ----------------------------------------------------------------------------
    def features(self, x):
        h = self.prepare_input(x)
        h = self.stem(h)
        h = self.layer4(self.layer3(self.layer2(self.layer1(h))))
        return self.avgpool(h)

    def forward_logits(self, x):
        f = self.features(x)
        if hasattr(self.fc, "forward_logits"):
            return self.fc.forward_logits(f)
        return self.fc(f)

    def forward(self, x):
        f = self.features(x)
        return self.fc(f)

    # ---- transfer learning ------------------------------------------------------------------
    def freeze_backbone(self):
        """another_neural_net.py:105-106 — every backbone param frozen; BN stays in train mode."""
        for n, p in self.named_parameters():
            if not n.startswith("fc."):
                p.requires_grad_(False)
        return self

    def replace_head(self, head: nn.Module):
        self.fc = head
        return self

    def backbone_modules(self):
        return [self.stem, self.layer1, self.layer2, self.layer3, self.layer4]

    # ---- pretrained weights ------------------------------------------------------------------
    @torch.no_grad()
    def load_torchvision(self, sd: dict, load_head: bool | None = None):
        """Load a torchvision-layout ResNet state_dict (``resnet50-19c8e357.pth``, the reference's
        ``models.resnet50(pretrained=True)``: nb :389,397-410, another_neural_net.py:95) or one saved
        from :class:`pcmp.models.torch_ref.TorchResNet`: KCRS conv weights -> KRSC (stem Cin padded to
        8), BN affine + running statistics, and the head when its shape matches (``fc.weight`` for a
        Linear, ``fc.0`` / ``fc.3`` for the reference's MLP head; ``load_head=False`` skips it, e.g.
        when a new TL head replaces the 1000-way fc).  Returns the list of state_dict keys used."""
        from .layers import Linear, MLPHead
        used = []

        def cbn(L, conv_key, bn_key):
            bn = {k: sd[f"{bn_key}.{k}"] for k in ("weight", "bias", "running_mean", "running_var")}
            w = sd[f"{conv_key}.weight"]
            assert tuple(w.shape) == (L.cout, L.cin, L.R, L.S), f"{conv_key}: {tuple(w.shape)} vs {(L.cout, L.cin, L.R, L.S)}"
            L.load_torch_conv_bn(w.to(L.weight.dtype), {k: v.to(L.gamma.dtype) for k, v in bn.items()})
            nbt = sd.get(f"{bn_key}.num_batches_tracked")
            if nbt is not None:
                L.num_batches_tracked.copy_(nbt)
            used.extend([f"{conv_key}.weight"] + [f"{bn_key}.{k}" for k in bn])

        cbn(self.stem.conv, "conv1", "bn1")
        for li, layer in enumerate([self.layer1, self.layer2, self.layer3, self.layer4], 1):
            for bi, blk in enumerate(layer):
                pre = f"layer{li}.{bi}"
                for ci, L in enumerate(blk.main_layers(), 1):
                    cbn(L, f"{pre}.conv{ci}", f"{pre}.bn{ci}")
                if blk.downsample is not None:
                    cbn(blk.downsample, f"{pre}.downsample.0", f"{pre}.downsample.1")

        def lin(L, key):
            w, b = sd.get(f"{key}.weight"), sd.get(f"{key}.bias")
            if w is None or tuple(w.shape) != (L.out_features, L.in_features):
                return False
            L.load_torch(w.to(L.weight.dtype), None if b is None else b.to(L.weight.dtype))
            used.extend([f"{key}.weight"] + ([f"{key}.bias"] if b is not None else []))
            return True

        if load_head is not False:
            if isinstance(self.fc, Linear):
                ok = lin(self.fc, "fc")
            elif isinstance(self.fc, MLPHead):
                ok = lin(self.fc.fc1, "fc.0") and lin(self.fc.fc2, "fc.3")
            else:
                ok = False
            if load_head and not ok:
                raise ValueError("load_torchvision: head weights missing or of another shape")
        for p in self.parameters():   # bf16 compute shadows of a flat arena follow the new masters
            owner = getattr(p, "_flat_owner", None)
            if owner is not None:
                owner.refresh_shadows()
                break
        return used


def resnet18(num_classes=1000, **kw):
    return ResNet("resnet18", num_classes, **kw)


def resnet34(num_classes=1000, **kw):
    return ResNet("resnet34", num_classes, **kw)


def resnet50(num_classes=1000, **kw):
    return ResNet("resnet50", num_classes, **kw)


def resnet101(num_classes=1000, **kw):
    return ResNet("resnet101", num_classes, **kw)


def resnet50_transfer(num_classes=10, hidden=512, p=0.2, **kw):
    """The reference's ResNet-50 TL model (another_neural_net.py:95-112)."""
    m = resnet50(1000, **kw).freeze_backbone()
    return m.replace_head(MLPHead(m.feature_dim, hidden, num_classes, p))


def count_params(model, logical=True):
    """Parameter count; ``logical`` subtracts the zero padding of Linear rows and stem channels."""
    total = 0
    for mod in model.modules():
        for name, p in mod.named_parameters(recurse=False):
            n = p.numel()
            if logical and isinstance(mod, Linear):
                n = n // mod.out_pad * mod.out_features if name == "weight" else mod.out_features
            elif logical and isinstance(mod, (ConvBN, Conv2d)) and name == "weight" and p.shape[-1] != mod.cin:
                n = n // p.shape[-1] * mod.cin
            total += n
    return total
