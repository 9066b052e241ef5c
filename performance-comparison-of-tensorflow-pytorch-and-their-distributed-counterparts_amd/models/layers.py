"""Framework layers: parameters in the layouts the HIP kernels consume.

* conv weights are KRSC ``[Cout, kh, kw, Cin]`` fp32 masters (bf16 compute shadow), activations
  NHWC;  Cin of the network input is zero-padded to a multiple of 8 (MFMA K granularity);
* Linear weights are ``[Nout_pad, Cin]`` with Nout padded to a multiple of 8 (the padding rows
  are zero and stay zero under SGD/Adam since their gradient is identically zero); the
  logical ``out_features`` is what the layer returns.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from ..ops.conv_blocks import ConvBiasActFn, GapFn, MaxPoolFn
from ..ops.functions import dropout, linear, log_softmax


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


class ConvBN(nn.Module):
    """Conv2d(bias=False) + BatchNorm2d parameters (executed by the fused block Functions).

    Initialisation follows torchvision's ResNet: kaiming_normal_(fan_out, relu) for the conv,
    gamma=1, beta=0 (``zero_init_gamma`` zeroes the last BN of a residual branch when asked).
    """

    def __init__(self, cin, cout, k, stride=1, pad=0, eps=1e-5, momentum=0.1, cin_pad=None,
                 zero_init_gamma=False):
        super().__init__()
        cin_p = cin_pad or cin
        self.cin, self.cout, self.R, self.S, self.stride, self.pad = cin, cout, k, k, stride, pad
        w = torch.empty(cout, cin, k, k)
        nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
        wk = torch.zeros(cout, k, k, cin_p)
        wk[..., :cin] = w.permute(0, 2, 3, 1)
        self.weight = nn.Parameter(wk)
        if stride == 2 and k > 1:
            # its DGRAD runs as four sub-pixel class GEMMs: the flat arena keeps the transposed
            # weight class-blocked for them (utils/flat.py)
            self.weight._pcmp_s2_pad = pad
        self.gamma = nn.Parameter(torch.zeros(cout) if zero_init_gamma else torch.ones(cout))
        self.beta = nn.Parameter(torch.zeros(cout))
        self.register_buffer("running_mean", torch.zeros(cout))
        self.register_buffer("running_var", torch.ones(cout))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self.eps, self.momentum = eps, momentum
        self.track_running_stats = True

    def params(self):
        return [self.weight, self.gamma, self.beta]

    def load_torch_conv_bn(self, conv_w: torch.Tensor, bn: dict):
        """Load torchvision-layout weights ([Cout,Cin,kh,kw] + BN dict)."""
        with torch.no_grad():
            self.weight.zero_()
            self.weight[..., : conv_w.shape[1]].copy_(conv_w.permute(0, 2, 3, 1))
            self.gamma.copy_(bn["weight"])
            self.beta.copy_(bn["bias"])
            self.running_mean.copy_(bn["running_mean"])
            self.running_var.copy_(bn["running_var"])


class Conv2d(nn.Module):
    """Conv2d(+bias)(+ReLU) with NHWC activations (VGG16 features)."""

    def __init__(self, cin, cout, k, stride=1, pad=0, bias=True, relu=False, cin_pad=None):
        super().__init__()
        cin_p = cin_pad or cin
        self.cin = cin
        self.R = self.S = k
        self.stride, self.pad, self.relu = stride, pad, relu
        w = torch.empty(cout, cin, k, k)
        nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
        wk = torch.zeros(cout, k, k, cin_p)
        wk[..., :cin] = w.permute(0, 2, 3, 1)
        self.weight = nn.Parameter(wk)
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None

    def forward(self, x):
        return ConvBiasActFn.apply(x, self, self.weight, self.bias)


class Linear(nn.Module):
    """y = act(x W^T + b) on the MFMA GEMM kernels; torch.nn.Linear default init."""

    def __init__(self, in_features, out_features, bias=True, relu=False):
        super().__init__()
        assert in_features % 8 == 0, "Linear in_features must be a multiple of 8"
        self.in_features, self.out_features, self.relu = in_features, out_features, relu
        self.out_pad = _pad8(out_features)
        w = torch.empty(out_features, in_features)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        wp = torch.zeros(self.out_pad, in_features)
        wp[:out_features] = w
        self.weight = nn.Parameter(wp)
        self.weight._pcmp_dgrad_t = True   # DGRAD reads a batched transposed shadow (utils/flat.py)
        if bias:
            bound = 1 / math.sqrt(in_features)
            b = torch.zeros(self.out_pad)
            b[:out_features].uniform_(-bound, bound)
            self.bias = nn.Parameter(b)
        else:
            self.bias = None

    def forward(self, x):
        shp = x.shape
        y = linear(x.reshape(-1, shp[-1]), self.weight, self.bias, self.relu)
        if self.out_pad != self.out_features:
            y = y[:, : self.out_features]
        return y.reshape(*shp[:-1], self.out_features)

    def load_torch(self, w, b=None):
        with torch.no_grad():
            self.weight.zero_()
            self.weight[: w.shape[0]].copy_(w)
            if b is not None and self.bias is not None:
                self.bias.zero_()
                self.bias[: b.shape[0]].copy_(b)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, relu={self.relu}"


class Dropout(nn.Module):
    def __init__(self, p):
        super().__init__()
        self.p = p

    def forward(self, x):
        return dropout(x, self.p, self.training)


class LogSoftmax(nn.Module):
    def forward(self, z):
        return log_softmax(z)


class MaxPool2d(nn.Module):
    def __init__(self, k, s, pad=0):
        super().__init__()
        self.k, self.s, self.pad = k, s, pad

    def forward(self, x):
        return MaxPoolFn.apply(x, self.k, self.s, self.pad)


class GlobalAvgPool(nn.Module):
    def forward(self, x):
        return GapFn.apply(x)


class MLPHead(nn.Module):
    """The reference's transfer-learning head:
    ``Linear(in,hidden)-ReLU-Dropout(p)-Linear(hidden,classes)[-LogSoftmax]``
    (another_neural_net.py:108-112 with (2048,512,0.2,10); :250-255 with (4096,256,0.4,10)).
    ``forward`` returns log-probabilities like the reference; ``forward_logits`` the logits used
    by the fused cross-entropy in training."""

    def __init__(self, in_features=2048, hidden=512, num_classes=10, p=0.2, log_softmax=True):
        super().__init__()
        self.fc1 = Linear(in_features, hidden, relu=True)
        self.drop = Dropout(p)
        self.fc2 = Linear(hidden, num_classes)
        self.emit_log_softmax = log_softmax

    def forward_logits(self, x):
        return self.fc2(self.drop(self.fc1(x)))

    def forward(self, x):
        z = self.forward_logits(x)
        return log_softmax(z) if self.emit_log_softmax else z
