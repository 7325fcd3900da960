"""Bucketed, backward-overlapped DDP (reference vendored ``ddp.py``)."""
from layer_wise_aaai20_amd.parallel.ddp import DistributedDataParallel  # noqa
