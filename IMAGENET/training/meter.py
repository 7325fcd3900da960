"""Meters (reference ``IMAGENET/training/meter.py``)."""
from layer_wise_aaai20_amd.utils.logging import (AverageMeter, NetworkMeter, TimeMeter,  # noqa
                                                 network_bytes)
