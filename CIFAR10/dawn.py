"""CIFAR-10 entry point (reference ``CIFAR10/dawn.py``): ``python -m CIFAR10.dawn --help``."""
import os
import sys

# runnable as a plain script (the reference launches ``training/train_imagenet_nv.py`` by path)
_ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from layer_wise_aaai20_amd.models.cifar import (alexnet, basic_alexnet, basic_resnet9, conv_bn,  # noqa
                                                conv_bn_stride, losses, residual, resnet9)
from layer_wise_aaai20_amd.train.cifar_main import get_parser, main  # noqa
from layer_wise_aaai20_amd.utils.logging import TSVLogger  # noqa

parser = get_parser()

if __name__ == "__main__":
    main(sys.argv[1:])
