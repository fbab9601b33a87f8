"""BNFusedHijacker (reference: quantization/quantized_folded_bn.py:15-95).

Same state machine as QuantizationHijacker, then F.batch_norm with the layer's own running
statistics (BN is applied after the approx product, not folded into the weights).
"""
import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.modules.conv import _ConvNd

from .hijacker import QuantizationHijacker


class BNFusedHijacker(QuantizationHijacker):
    def __init__(self, *args, **kwargs):
        kwargs.pop("bias", None)
        super().__init__(*args, **kwargs, bias=False)
        dim = self.get_bn_dim()
        self.register_buffer("running_mean", torch.zeros(dim))
        self.register_buffer("running_var", torch.ones(dim))
        self.momentum = kwargs.pop("momentum", 0.1)
        self.gamma = nn.Parameter(torch.ones(dim))
        self.beta = nn.Parameter(torch.zeros(dim))
        self.epsilon = kwargs.get("eps", 1e-5)
        self.bias = None

    def forward(self, x):
        res, qa = self._core(x)
        res = F.batch_norm(res, self.running_mean, self.running_var, self.gamma, self.beta, self.training,
                           self.momentum, self.epsilon)
        return self._epilogue(res, qa)

    def get_bn_dim(self):
        if isinstance(self, nn.Linear):
            return self.out_features
        if isinstance(self, _ConvNd):
            return self.out_channels
        raise NotImplementedError(f"Unsupported type used: {self}. Must be a linear or convolutional nn.Module")
