"""Reference-layout compatibility package: ``CIFAR10.core`` / ``CIFAR10.torch_backend`` /
``CIFAR10.dawn`` / ``CIFAR10.alexnet`` / ``CIFAR10.vgg16`` re-export the MI355X-native
implementations in :mod:`layer_wise_aaai20_amd`."""
