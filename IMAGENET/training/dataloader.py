"""``IMAGENET.training.dataloader`` (synthetic ImageNet; see layer_wise_aaai20_amd.data.imagenet)."""
from layer_wise_aaai20_amd.data.imagenet import (BatchTransformDataLoader, DistValSampler,  # noqa
                                                 RectValDataset, SyntheticImageNet, chunks,
                                                 crop_size_for_ar, fast_collate, get_loaders,
                                                 map_idx2ar, sort_ar)
