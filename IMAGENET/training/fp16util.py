"""fp16 helpers (reference ``IMAGENET/training/fp16util.py``)."""
from layer_wise_aaai20_amd.utils.fp16 import (BN_convert_float, backwards_debug_hook,  # noqa
                                              master_params_to_model_params,
                                              model_grads_to_master_grads, network_to_half,
                                              prep_param_lists, tofp16)
