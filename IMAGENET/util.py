"""Launcher utilities (reference ``IMAGENET/util.py``). Config transport is base64 JSON: nothing is
unpickled."""
from layer_wise_aaai20_amd.utils.launch import (environment_snapshot, format_env, is_set,  # noqa
                                                log_environment, ossystem, random_id,
                                                text_decode, text_encode)

text_pickle = text_encode
text_unpickle = text_decode
