"""Decode heads (reference seg/denseclip/heads.py and the torchvision FCNHead the reference
builds for 'FPNHead' / 'FCNHeadDepth', denseclip.py:22-23, 305-309, 343-349)."""
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .models import BatchNorm2d, Registry


class FCNHead(nn.Sequential):
    """torchvision.models.segmentation.fcn.FCNHead: conv3x3(in -> in/4, no bias), BN, ReLU,
    Dropout(0.1), conv1x1(in/4 -> channels).  DenseCLIP then assigns a `.classifier`
    conv, which nn.Sequential appends to the module sequence (so it runs last).

    On a 16-bit GPU map the forward runs on the HIP kernels (ops.fcn_head): the 3x3 conv as an
    implicit GEMM, BN + ReLU fused, and the two trailing 1x1 convs merged into one GEMM
    (ops.MergedPointwiseFn) — same parameters, same function."""

    def __init__(self, in_channels, channels):
        inter = in_channels // 4
        super().__init__(
            nn.Conv2d(in_channels, inter, 3, padding=1, bias=False),
            BatchNorm2d(inter),
            nn.ReLU(),
            nn.Dropout(0.1),
            nn.Conv2d(inter, channels, 1),
        )

    def forward(self, x):
        if ops.fcn_head_hip_ok(self, x):
            return ops.fcn_head(self, x)
        ops.note_torch_fallback()
        return super().forward(x)


class ConvModule(nn.Module):
    """mmcv ConvModule replacement (reference heads.py:7-48)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 bias=True, norm_cfg=None, act_cfg=None):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                              dilation=dilation, groups=groups, bias=bias)
        self.norm = BatchNorm2d(out_channels) if norm_cfg is not None else None
        self.activate = nn.ReLU(inplace=True) if act_cfg is not None else None

    def forward(self, x):
        x = self.conv(x)
        if self.norm is not None:
            x = self.norm(x)
        if self.activate is not None:
            x = self.activate(x)
        return x


def resize(input, size=None, scale_factor=None, mode="bilinear", align_corners=None):
    return F.interpolate(input, size=size, scale_factor=scale_factor, mode=mode, align_corners=align_corners)


HEADS = Registry()


class BaseDecodeHead(nn.Module):
    def __init__(self, input_transform=None, **kwargs):
        super().__init__()
        self.input_transform = input_transform

    def forward(self, inputs):
        raise NotImplementedError


@HEADS.register_module()
class IdentityHead(BaseDecodeHead):
    """Returns its input (reference heads.py:81-106)."""

    def __init__(self, **kwargs):
        super().__init__(input_transform=None, **kwargs)
        self.conv_seg = None

    def forward(self, inputs):
        return inputs
