"""ResNet family (reference ``IMAGENET/training/resnet.py``)."""
from layer_wise_aaai20_amd.models.resnet import (BasicBlock, Bottleneck, ResNet, conv3x3,  # noqa
                                                 init_dist_weights, resnet18, resnet34, resnet50,
                                                 resnet101, resnet152)
