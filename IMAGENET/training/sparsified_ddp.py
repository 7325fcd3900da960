"""Shared-seed Random-K sparsified DDP with error feedback (reference ``sparsified_ddp.py``)."""
from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP, RandomKSparsifiedDDP  # noqa
