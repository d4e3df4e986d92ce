"""CLIP ModifiedResNet image tower + preprocessing (reference ``model/image_encoder/clip.py``).

Module / parameter names match the reference so checkpoints load unchanged.  Preprocessing is done
with PIL + torch (torchvision is not part of the ROCm image): bicubic resize of the short side,
center crop, RGB, [0, 1] tensor, CLIP mean/std normalisation.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable

import numpy as np
import torch
from PIL import Image

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def convert_image_to_rgb(image: Image.Image) -> Image.Image:
    return image.convert("RGB")


def clip_transform(n_px: tuple[int, int]) -> Callable[[Image.Image], torch.Tensor]:
    th, tw = n_px
    mean = torch.tensor(CLIP_MEAN).view(3, 1, 1)
    std = torch.tensor(CLIP_STD).view(3, 1, 1)

    def transform(image: Image.Image) -> torch.Tensor:
        w, h = image.size
        # Resize(tuple) resizes to exactly (h, w) = n_px
        image = image.resize((tw, th), resample=Image.BICUBIC)
        w, h = image.size
        left, top = int(round((w - tw) / 2.0)), int(round((h - th) / 2.0))
        image = image.crop((left, top, left + tw, top + th))
        arr = np.asarray(convert_image_to_rgb(image), dtype=np.float32) / 255.0
        t = torch.from_numpy(arr).permute(2, 0, 1).contiguous()
        return (t - mean) / std

    return transform


def _conv_bn(cin: int, cout: int, k: int, **kw: int) -> tuple[torch.nn.Conv2d, torch.nn.BatchNorm2d]:
    return torch.nn.Conv2d(cin, cout, k, bias=False, **kw), torch.nn.BatchNorm2d(cout)


class Bottleneck(torch.nn.Module):
    """1x1 → 3x3 → (avgpool when strided) → 1x1 bottleneck; anti-aliased strided shortcut."""

    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1) -> None:
        super().__init__()
        width_out = planes * self.expansion
        self.conv1, self.bn1 = _conv_bn(inplanes, planes, 1)
        self.conv2, self.bn2 = _conv_bn(planes, planes, 3, padding=1)
        self.avgpool = torch.nn.AvgPool2d(stride) if stride > 1 else torch.nn.Identity()
        self.conv3, self.bn3 = _conv_bn(planes, width_out, 1)
        self.relu = torch.nn.ReLU(inplace=True)
        self.stride = stride
        self.downsample = None
        if stride > 1 or inplanes != width_out:
            conv, bn = _conv_bn(inplanes, width_out, 1, stride=1)
            self.downsample = torch.nn.Sequential(OrderedDict([("-1", torch.nn.AvgPool2d(stride)), ("0", conv), ("1", bn)]))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.avgpool(self.relu(self.bn2(self.conv2(y))))
        y = self.bn3(self.conv3(y))
        y += x if self.downsample is None else self.downsample(x)
        return self.relu(y)


class ClipModifiedResNet(torch.nn.Module):
    """3-conv stem + avgpool, four bottleneck stages; returns the final feature map as tokens [b, h*w, d]."""

    def __init__(self, layers: list[int], num_init_channels: int = 64):
        super().__init__()
        c = num_init_channels
        self.conv1, self.bn1 = _conv_bn(3, c // 2, 3, stride=2, padding=1)
        self.conv2, self.bn2 = _conv_bn(c // 2, c // 2, 3, padding=1)
        self.conv3, self.bn3 = _conv_bn(c // 2, c, 3, padding=1)
        self.avgpool = torch.nn.AvgPool2d(2)
        self.relu = torch.nn.ReLU(inplace=True)
        self._inplanes = c
        self.layer1 = self._make_layer(c, layers[0])
        self.layer2 = self._make_layer(2 * c, layers[1], stride=2)
        self.layer3 = self._make_layer(4 * c, layers[2], stride=2)
        self.layer4 = self._make_layer(8 * c, layers[3], stride=2)

    def _make_layer(self, planes: int, blocks: int, stride: int = 1) -> torch.nn.Sequential:
        mods = [Bottleneck(self._inplanes, planes, stride)]
        self._inplanes = planes * Bottleneck.expansion
        mods += [Bottleneck(self._inplanes, planes) for _ in range(1, blocks)]
        return torch.nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.type(self.conv1.weight.dtype)
        for conv, bn in ((self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)):
            x = self.relu(bn(conv(x)))
        x = self.avgpool(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        b, d, h, w = x.shape
        return x.reshape(b, d, h * w).transpose(1, 2)
