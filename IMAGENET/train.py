"""Job launcher (reference ``IMAGENET/train.py``): ``python -m IMAGENET.train --help``."""
import sys

from layer_wise_aaai20_amd.train.launcher import get_parser, main  # noqa
from layer_wise_aaai20_amd.train.schedules import schedules  # noqa
from layer_wise_aaai20_amd.utils.launch import build_ring_order, get_rings, get_skip_order  # noqa

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
