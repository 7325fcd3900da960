"""Loggers (reference ``IMAGENET/training/logger.py``)."""
from layer_wise_aaai20_amd.utils.logging import FileLogger, NoOp, TensorboardLogger  # noqa
