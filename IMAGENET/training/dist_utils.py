"""``dist_utils`` (reference ``IMAGENET/training/dist_utils.py``)."""
from layer_wise_aaai20_amd.parallel.comm import (env_rank, env_world_size, reduce_tensor,  # noqa
                                                 sum_tensor)
from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP as DDP  # noqa
