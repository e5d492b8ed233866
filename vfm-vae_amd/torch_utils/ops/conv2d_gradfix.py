"""`conv2d` / `conv_transpose2d` with the reference's gradfix switches.

The reference module (`torch_utils/ops/conv2d_gradfix.py:22-58`) installs a
custom autograd op only for torch < 1.11; on every torch this package supports
it is a pass-through to `torch.nn.functional`. The switches (`enabled`,
`weight_gradients_disabled`, `no_weight_gradients()`) are kept so callers that
toggle them (reference training_loop.py:506) keep working.
"""
import contextlib

import torch

enabled = False
weight_gradients_disabled = False


@contextlib.contextmanager
def no_weight_gradients(disable=True):
    global weight_gradients_disabled
    previous = weight_gradients_disabled
    if disable:
        weight_gradients_disabled = True
    try:
        yield
    finally:
        weight_gradients_disabled = previous


def conv2d(input, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    return torch.nn.functional.conv2d(input=input, weight=weight, bias=bias, stride=stride,
                                      padding=padding, dilation=dilation, groups=groups)


def conv_transpose2d(input, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1):
    return torch.nn.functional.conv_transpose2d(input=input, weight=weight, bias=bias, stride=stride,
                                                padding=padding, output_padding=output_padding,
                                                groups=groups, dilation=dilation)
