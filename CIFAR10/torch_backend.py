"""``CIFAR10.torch_backend`` API (reference ``CIFAR10/torch_backend.py``) on layer_wise_aaai20_amd."""
import numpy as np
import torch

from layer_wise_aaai20_amd.data.cifar import Batches, GPUBatches, cifar10, synthetic_cifar10  # noqa
from layer_wise_aaai20_amd.models.graph import (SGD, Add, Concat, Correct, Flatten, Identity,  # noqa
                                                Mul, Network, TorchOptimiser, batch_norm,
                                                trainable_params)
from layer_wise_aaai20_amd.utils.viz import cat, to_numpy  # noqa

torch.backends.cudnn.benchmark = True   # MIOpen find mode on ROCm
device = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")


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
