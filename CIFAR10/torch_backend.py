"""``CIFAR10.torch_backend`` API (reference ``CIFAR10/torch_backend.py``) on layer_wise_aaai20_amd."""
import numpy as np
import torch

from layer_wise_aaai20_amd.data.cifar import Batches, GPUBatches, cifar10, synthetic_cifar10  # noqa
from layer_wise_aaai20_amd.models.graph import (SGD, Add, Concat, Correct, Flatten, Identity,  # noqa
                                                Mul, Network, TorchOptimiser, batch_norm,
                                                trainable_params)
from layer_wise_aaai20_amd.utils.viz import cat, to_numpy  # noqa

torch.backends.cudnn.benchmark = True   # MIOpen find mode on ROCm
def _rank_device() -> torch.device:
    """This rank's GPU (``cuda:LOCAL_RANK``, else ``RANK % device_count``); the reference pins
    every rank to ``cuda:0`` (``torch_backend.py:8``), which puts a one-node world on one GPU."""
    if not torch.cuda.is_available():
        return torch.device("cpu")
    from layer_wise_aaai20_amd.parallel.comm import env_local_rank, env_rank, rank_device_index
    return torch.device("cuda", rank_device_index(env_rank(), torch.cuda.device_count(),
                                                  env_local_rank()))


device = _rank_device()


def warmup_cudnn(model, batch_size, dev=None):
    """One forward+backward on a random batch so MIOpen benchmarks its conv solvers up front
    (reference ``torch_backend.py:18-29``)."""
    dev = dev or device
    if batch_size <= 0:
        return
    batch = {"input": torch.tensor(np.random.rand(batch_size, 3, 32, 32), dtype=torch.float32,
                                   device=dev),
             "target": torch.tensor(np.random.randint(0, 10, batch_size), dtype=torch.long,
                                    device=dev)}
    model.train(True)
    out = model(batch)
    out["loss"].sum().backward()
    model.zero_grad()
    if dev.type == "cuda":
        torch.cuda.synchronize()
