"""The TensorFlow/Keras counterpart of the reference (resnet.py), re-expressed on the HIP path.

resnet.py:17-24: ``ResNet50(weights='imagenet', include_top=False, input_shape=(224,224,3))`` ->
``Flatten`` (7*7*2048 = 100,352 features) -> ``Dense(num_classes, activation='softmax')``;
compiled with ``SGD(lr=0.001)`` and ``categorical_crossentropy``; the backbone is NOT frozen (full
fine-tune).  Keras ResNet50 v1 puts the downsampling stride on the first 1x1 convolution
(``variant='keras'``).  The "single HIP path" north star excludes a TF backend, so this is the same
framework with Keras semantics: one-hot (categorical) targets, softmax output, Keras image
preprocessing (``rescale=1./255`` of ImageDataGenerator, resnet.py:11; or caffe-style
``preprocess_input``: RGB->BGR and ImageNet mean subtraction).
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops.functions import cross_entropy, log_softmax
from .layers import Linear
from .resnet import ResNet

CAFFE_MEAN_BGR = (103.939, 116.779, 123.68)


class KerasResNet50TL(nn.Module):
    def __init__(self, num_classes=10, compute_dtype=None, image_size=224):
        super().__init__()
        self.backbone = ResNet("resnet50", 1000, variant="keras", compute_dtype=compute_dtype)
        self.backbone.fc = nn.Identity()
        fm = (image_size + 31) // 32                       # 7 at 224
        self.dense = Linear(fm * fm * 2048, num_classes)  # "transfer_lr" Dense (100,352 inputs at 224)
        self.num_classes = num_classes

    def forward_logits(self, x):
        bb = self.backbone
        h = bb.prepare_input(x)
        h = bb.stem(h)
        h = bb.layer4(bb.layer3(bb.layer2(bb.layer1(h))))
        return self.dense(h.reshape(h.shape[0], -1))      # Flatten in NHWC order

    def forward(self, x):
        """softmax probabilities (Keras Dense activation='softmax')."""
        return torch.exp(log_softmax(self.forward_logits(x)))


def categorical_crossentropy(logits, onehot):
    """Keras categorical CE on one-hot targets (the integer-label fused kernel underneath)."""
    return cross_entropy(logits, onehot.argmax(1))


def preprocess_rescale(x_uint8_nhwc: torch.Tensor) -> torch.Tensor:
    """ImageDataGenerator(rescale=1./255) on NHWC uint8 -> NCHW float."""
    return (x_uint8_nhwc.float() / 255.0).permute(0, 3, 1, 2).contiguous()


def preprocess_input_caffe(x_rgb_nhwc: torch.Tensor) -> torch.Tensor:
    """keras.applications.resnet50.preprocess_input ('caffe'): RGB->BGR, subtract ImageNet mean."""
    x = x_rgb_nhwc.float()[..., [2, 1, 0]]
    x = x - torch.tensor(CAFFE_MEAN_BGR, device=x.device)
    return x.permute(0, 3, 1, 2).contiguous()
