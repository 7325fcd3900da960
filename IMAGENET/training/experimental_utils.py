"""No-BN-weight-decay parameter groups (reference ``experimental_utils.py``), without the
same-generator-zipped-with-itself bug of the fp32 path."""
import torch


def split_bn_params(model, model_params, master_params):
    bn = set()
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            bn.update(id(p) for p in m.parameters())
    pairs = list(zip(list(model_params), list(master_params)))
    return ([mp for p, mp in pairs if id(p) in bn], [mp for p, mp in pairs if id(p) not in bn])


def bnwd_optim_params(model, model_params, master_params):
    model_params = list(model_params)
    master_params = list(master_params) if master_params is not None else model_params
    if len(master_params) != len(model_params):   # one generator passed twice (D12)
        master_params = model_params
    bn_params, rest = split_bn_params(model, model_params, master_params)
    return [{"params": bn_params, "weight_decay": 0}, {"params": rest}]
