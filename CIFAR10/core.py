"""``CIFAR10.core`` API (reference ``CIFAR10/core.py``) on layer_wise_aaai20_amd."""
from layer_wise_aaai20_amd.data.cifar import (Crop, Cutout, FlipLR, Transform, cifar10_mean,  # noqa
                                              cifar10_std, normalise, pad, transpose)
from layer_wise_aaai20_amd.models.graph import (RelativePath, build_graph, path_iter, rel_path,  # noqa
                                                sep, union)
from layer_wise_aaai20_amd.parallel.functional import (all_reduce, compressed_comm,  # noqa
                                                       entiremodel_compressed_comm,
                                                       layerwise_compressed_comm)
from layer_wise_aaai20_amd.train.cifar import run_batches, train, train_epoch  # noqa
from layer_wise_aaai20_amd.utils.logging import (PiecewiseLinear, StatsLogger, TableLogger,  # noqa
                                                 Timer, localtime)
from layer_wise_aaai20_amd.utils.viz import (ColorMap, DotGraph, cat, get_params,  # noqa
                                             remove_by_type, to_numpy, walk)
