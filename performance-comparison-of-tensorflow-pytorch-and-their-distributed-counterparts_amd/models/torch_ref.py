"""Plain ``torch.nn`` re-statements of the framework's models.

Two uses:
  1. numerics parity: ``TorchResNet.from_pcmp(model)`` copies a framework model's weights into a
     stock nn.Conv2d/nn.BatchNorm2d network so tests compare loss and gradients;
  2. the **self-baseline** of ``bench.py --impl torch``: the same architecture run on stock
     PyTorch-ROCm (MIOpen convolutions, channels_last, bf16 autocast) on the same MI355X.
torchvision is not installed in this image, so the topology is written out here (it follows
the printout at pytorch_training_inference_on_image.ipynb:454-635).
"""
from __future__ import annotations

import torch
from torch import nn


class TBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride, stride_in_1x1=False):
        super().__init__()
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = nn.Conv2d(cin, planes, 1, s1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, s3, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != planes * 4:
            self.downsample = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride, bias=False),
                                            nn.BatchNorm2d(planes * 4))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class TBasic(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride, stride_in_1x1=False):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != planes:
            self.downsample = nn.Sequential(nn.Conv2d(cin, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


_CFG = {"resnet18": (TBasic, [2, 2, 2, 2]), "resnet34": (TBasic, [3, 4, 6, 3]),
        "resnet50": (TBottleneck, [3, 4, 6, 3]), "resnet101": (TBottleneck, [3, 4, 23, 3])}


class TorchResNet(nn.Module):
    def __init__(self, arch="resnet50", num_classes=1000, head=None, stride_in_1x1=False):
        super().__init__()
        block, layers = _CFG[arch]
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        stages = []
        for i, (planes, n) in enumerate(zip([64, 128, 256, 512], layers)):
            blocks = []
            for j in range(n):
                blocks.append(block(cin, planes, 2 if (j == 0 and i > 0) else 1, stride_in_1x1))
                cin = planes * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = head if head is not None else nn.Linear(cin, num_classes)
        # torchvision ResNet initialisation (the reference's models.resnet50): kaiming-normal
        # fan_out convs, BN gamma=1 / beta=0; Linear keeps the nn.Linear default.
        for mod in self.modules():
            if isinstance(mod, nn.Conv2d):
                nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(mod, nn.BatchNorm2d):
                nn.init.ones_(mod.weight)
                nn.init.zeros_(mod.bias)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    @torch.no_grad()
    def load_from_pcmp(self, m):
        """Copy weights (KRSC -> KCRS) and BN state from a framework ResNet."""
        from .layers import Linear, MLPHead

        def cp_cbn(conv, bn, L):
            conv.weight.copy_(L.weight[..., : conv.weight.shape[1]].permute(0, 3, 1, 2))
            bn.weight.copy_(L.gamma)
            bn.bias.copy_(L.beta)
            bn.running_mean.copy_(L.running_mean)
            bn.running_var.copy_(L.running_var)

        cp_cbn(self.conv1, self.bn1, m.stem.conv)
        for tl, pl in zip([self.layer1, self.layer2, self.layer3, self.layer4],
                          [m.layer1, m.layer2, m.layer3, m.layer4]):
            for tb, pb in zip(tl, pl):
                names = ["1", "2", "3"][: len(pb.main_layers())]
                for nm, L in zip(names, pb.main_layers()):
                    cp_cbn(getattr(tb, "conv" + nm), getattr(tb, "bn" + nm), L)
                if pb.downsample is not None:
                    cp_cbn(tb.downsample[0], tb.downsample[1], pb.downsample)

        def cp_lin(t, p):
            t.weight.copy_(p.weight[: p.out_features])
            if t.bias is not None:
                t.bias.copy_(p.bias[: p.out_features])

        if isinstance(m.fc, Linear):
            cp_lin(self.fc, m.fc)
        elif isinstance(m.fc, MLPHead):
            cp_lin(self.fc[0], m.fc.fc1)
            cp_lin(self.fc[3], m.fc.fc2)
        return self


def torch_mlp_head(in_features=2048, hidden=512, num_classes=10, p=0.2):
    return nn.Sequential(nn.Linear(in_features, hidden), nn.ReLU(), nn.Dropout(p),
                         nn.Linear(hidden, num_classes), nn.LogSoftmax(dim=1))


def grads_of_pcmp_block_order(tm: TorchResNet):
    """Flatten (name, grad) pairs in the framework's parameter order for comparisons."""
    return {n: p.grad for n, p in tm.named_parameters()}
