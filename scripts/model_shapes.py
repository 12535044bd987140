"""State_dict layouts of the reference's BASELINE models (FedML architectures;
FedML itself is absent from /root/reference, so these are reconstructed from
the architectures main_fedavg.py:237-270 selects).  Used to build synthetic
client updates of the right key structure for the benchmarks and the CPU
baseline; the product path never imports this.
"""
from __future__ import annotations

import math


def resnet56_shapes(num_classes=10):
    """FedML resnet56 (Bottleneck, [6, 6, 6]) state_dict: 350 keys, 600,372 elements."""
    shapes = []

    def bn(prefix, c):
        shapes.extend([(f"{prefix}.weight", (c,)), (f"{prefix}.bias", (c,)), (f"{prefix}.running_mean", (c,)),
                       (f"{prefix}.running_var", (c,)), (f"{prefix}.num_batches_tracked", ())])

    shapes.append(("conv1.weight", (16, 3, 3, 3)))
    bn("bn1", 16)
    inplanes = 16
    for li, (planes, stride) in enumerate([(16, 1), (32, 2), (64, 2)], 1):
        for b in range(6):
            p = f"layer{li}.{b}"
            shapes.append((f"{p}.conv1.weight", (planes, inplanes, 1, 1)))
            bn(f"{p}.bn1", planes)
            shapes.append((f"{p}.conv2.weight", (planes, planes, 3, 3)))
            bn(f"{p}.bn2", planes)
            shapes.append((f"{p}.conv3.weight", (planes * 4, planes, 1, 1)))
            bn(f"{p}.bn3", planes * 4)
            if b == 0 and (stride != 1 or inplanes != planes * 4):
                shapes.append((f"{p}.downsample.0.weight", (planes * 4, inplanes, 1, 1)))
                bn(f"{p}.downsample.1", planes * 4)
            inplanes = planes * 4
    shapes.append(("fc.weight", (num_classes, 256)))
    shapes.append(("fc.bias", (num_classes,)))
    return shapes


def resnet18_gn_shapes(num_classes=100):
    """FedML resnet18_gn for fed_cifar100 (BasicBlock [2, 2, 2, 2], 7x7 stem,
    GroupNorm: weight + bias, no running statistics): 62 keys, 11,227,812
    elements."""
    shapes = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    inplanes = 64
    for li, (planes, stride) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)], 1):
        for b in range(2):
            p = f"layer{li}.{b}"
            shapes += [(f"{p}.conv1.weight", (planes, inplanes, 3, 3)), (f"{p}.bn1.weight", (planes,)),
                       (f"{p}.bn1.bias", (planes,)), (f"{p}.conv2.weight", (planes, planes, 3, 3)),
                       (f"{p}.bn2.weight", (planes,)), (f"{p}.bn2.bias", (planes,))]
            if b == 0 and (stride != 1 or inplanes != planes):
                shapes += [(f"{p}.downsample.0.weight", (planes, inplanes, 1, 1)),
                           (f"{p}.downsample.1.weight", (planes,)), (f"{p}.downsample.1.bias", (planes,))]
            inplanes = planes
    shapes += [("fc.weight", (num_classes, 512)), ("fc.bias", (num_classes,))]
    return shapes


CONFIGS = {
    "mnist_lr": (10, [("linear.weight", (10, 784)), ("linear.bias", (10,))]),
    "femnist_cnn": (10, [("conv2d_1.weight", (32, 1, 3, 3)), ("conv2d_1.bias", (32,)),
                         ("conv2d_2.weight", (64, 32, 3, 3)), ("conv2d_2.bias", (64,)),
                         ("linear_1.weight", (128, 9216)), ("linear_1.bias", (128,)),
                         ("linear_2.weight", (62, 128)), ("linear_2.bias", (62,))]),
    "resnet56": (100, resnet56_shapes()),
    "resnet18_gn": (500, resnet18_gn_shapes()),
    "target_flat": (100, [("w", (25_000_000,))]),
    "flat_640x3m": (640, [("w", (3_000_000,))]),      # split-row zero-copy windows, 16 waves
    "flat_1000x5m": (1000, [("w", (5_000_000,))]),
    "flat_300x5m": (300, [("w", (5_000_000,))]),
    "flat_260x8m": (260, [("w", (8_000_000,))]),
    "flat_320x3m": (320, [("w", (3_000_000,))]),
    # resnet56's fp32 element count as ONE key (tile / window probes: the
    # per-key cost against the same bytes)
    "resnet56_flat": (100, [("w", (600_372 - 58,))]),
}


def numel(shapes) -> int:
    return sum(math.prod(s) for _, s in shapes)
