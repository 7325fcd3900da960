"""``CIFAR10.alexnet`` (reference ``CIFAR10/alexnet.py``)."""
from layer_wise_aaai20_amd.models.cifar import AlexNet  # noqa

NUM_CLASSES = 10
