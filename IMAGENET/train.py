"""Job launcher (reference ``IMAGENET/train.py``): ``python -m IMAGENET.train --help``."""
import os
import sys

# runnable as a plain script (the reference launches ``training/train_imagenet_nv.py`` by path)
_ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from layer_wise_aaai20_amd.train.launcher import get_parser, main  # noqa
from layer_wise_aaai20_amd.train.schedules import schedules  # noqa
from layer_wise_aaai20_amd.utils.launch import build_ring_order, get_rings, get_skip_order  # noqa

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
