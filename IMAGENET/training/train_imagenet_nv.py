"""ImageNet entry point (reference ``IMAGENET/training/train_imagenet_nv.py``)."""
import os
import sys

# runnable as a plain script (the reference launches ``training/train_imagenet_nv.py`` by path)
_ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from layer_wise_aaai20_amd.parallel.functional import (all_reduce,  # noqa
                                                       entiremodel_compressed_comm,
                                                       layerwise_compressed_comm)
from layer_wise_aaai20_amd.train.imagenet_main import (DataManager, Scheduler, accuracy,  # noqa
                                                       correct, distributed_predict, get_parser,
                                                       listify, main, save_checkpoint,
                                                       to_python_float, train, validate)

if __name__ == "__main__":
    main(sys.argv[1:])
