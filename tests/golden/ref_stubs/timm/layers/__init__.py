import torch.nn as nn


def trunc_normal_(tensor, mean=0., std=1., a=-2., b=2.):
    return nn.init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


def get_norm_layer(name):
    assert name == 'layernorm'
    return nn.LayerNorm
