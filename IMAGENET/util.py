"""Launcher utilities (reference ``IMAGENET/util.py``). Config transport is base64 JSON: nothing is
unpickled."""
from layer_wise_aaai20_amd.utils.launch import (environment_snapshot, format_env,  # noqa
                                                format_env_export, get_nccl_params, is_set,
                                                log_environment, mount_imagenet, ossystem,
                                                random_id, run_parallel, setup_mpi, text_decode,
                                                text_encode)

text_pickle = text_encode
text_unpickle = text_decode
