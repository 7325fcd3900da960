"""Reference-layout compatibility package for the ImageNet workload."""
