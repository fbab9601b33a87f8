"""Model-level wiring of the approx operators: the module swap and the quantized-model switches.

Restates the behaviour of the reference's approx/replace_operations_with_approx_ops.py
(fold_bn :263-286, quantize_sequential :289-342, quantize_model :345-384, the module maps
:180-193) and quantization/base_quantized_model.py (QuantizedModel switches :19-139), plus
autoquant_utils.QuantizedActivationWrapper / Flattener (:125-181): which layers of a float
model become approx operators, with which activation folded in, and how pooling layers tie
their output quantizer to the preceding layer's.  A float model passed through
``quantize_model`` gets the same module tree (and state_dict keys) as with the reference.

Only the approx path is mapped: Conv2d (+BN) -> QCustomBNConv2dTorch, Conv2d without BN ->
QCustomConv2dTorch (exact product, as in the reference), Linear -> QCustomLinearTorch, and
LayerNorm -> QuantLayerNorm (the ViT caller's norms).  The reference's other non-approx
quantized layers (Conv1d, ConvTranspose, Linear + BN) are outside the hot path and
raise NotImplementedError here.
"""
import os
import copy
import warnings

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.modules.conv import _ConvNd
from torch.nn.modules.pooling import _AdaptiveAvgPoolNd, _AvgPoolNd

from . import chain
from .approx_calculation import QCustomBNConv2dTorch, QCustomConv2dTorch, QCustomLinearTorch
from .quantization.base_quantized_classes import (QuantizedActivation, QuantizedModule, _set_layer_approx_calculation,
                                                  _set_layer_estimate_ranges, _set_layer_fix_ranges)
from .quantization.hijacker import QuantizationHijacker, activations_set
from .quantization.quantization_manager import QuantizationManager

__all__ = ["QuantizedModel", "QuantizedActivationWrapper", "Flattener", "QuantLayerNorm", "fold_bn",
           "quantize_sequential", "quantize_model", "non_bn_module_map", "bn_module_map"]



class QuantLayerNorm(QuantizationHijacker, nn.LayerNorm):
    """autoquant_utils.py:166-174: FP8-quantized input and (per-channel) weight, then a plain
    fp32 layer norm -- not an approx product."""

    def run_forward(self, x, weight, bias, offsets=None):
        return F.layer_norm(x.contiguous(), self.normalized_shape, weight.contiguous(), bias.contiguous(), self.eps)


non_bn_module_map = {nn.Conv2d: QCustomConv2dTorch, nn.Linear: QCustomLinearTorch, nn.LayerNorm: QuantLayerNorm}
bn_module_map = {nn.Conv2d: QCustomBNConv2dTorch}
non_param_modules = (_AdaptiveAvgPoolNd, _AvgPoolNd)
_OFF_PATH = (nn.Conv1d, nn.ConvTranspose1d, nn.ConvTranspose2d)


class QuantizedModel(nn.Module):
    """Whole-model quantization switches (base_quantized_model.py:19-139)."""

    def __init__(self, input_size=(1, 3, 224, 224)):
        super().__init__()
        self.input_size = input_size

    def _each(self, name):
        def fn(layer):
            if isinstance(layer, QuantizedModule):
                getattr(layer, name)()
        self.apply(fn)

    def quantized_weights(self):
        self._each("quantized_weights")

    def full_precision_weights(self):
        self._each("full_precision_weights")

    def quantized_acts(self):
        self._each("quantized_acts")

    def full_precision_acts(self):
        self._each("full_precision_acts")

    def quantized(self):
        self._each("quantized")

    def full_precision(self):
        self._each("full_precision")

    def set_quant_state(self, weight_quant, act_quant):
        (self.quantized_acts if act_quant else self.full_precision_acts)()
        (self.quantized_weights if weight_quant else self.full_precision_weights)()

    def estimate_ranges(self):
        self.apply(_set_layer_estimate_ranges)

    def fix_ranges(self):
        self.apply(_set_layer_fix_ranges)

    def approx_calculation(self):
        self.apply(_set_layer_approx_calculation)

    def load_state_dict(self, state_dict, strict=True):
        """The reference loads the quantization on/off states first and runs one dummy forward
        so lazily-shaped quantizer tensors exist before the full load
        (base_quantized_model.py:35-63)."""
        quant = {k: v for k, v in state_dict.items() if k.endswith("_quant_a") or k.endswith("_quant_w")}
        if not quant:
            raise ValueError("The quantization states of activations or weights should be included in the state dict ")
        super().load_state_dict(quant, strict=False)
        device = next(self.parameters()).device
        with torch.no_grad():
            self.forward(torch.rand(*self.input_size, device=device))
        return super().load_state_dict(state_dict, strict)


class QuantizedActivationWrapper(QuantizedActivation):
    """A parameter-free layer followed by an activation quantizer, optionally the preceding
    layer's quantizer used without range update (autoquant_utils.py:125-163)."""

    def __init__(self, layer, tie_activation_quantizers=False, input_quantizer=None, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.tie_activation_quantizers = tie_activation_quantizers
        if input_quantizer:
            assert isinstance(input_quantizer, QuantizationManager)
            self.activation_quantizer = input_quantizer
        self.layer = layer

    def quantize_activations_no_range_update(self, x):
        return self.activation_quantizer.quantizer(x) if self._qa() else x

    def forward(self, x):
        x = self.layer(x)
        if self.tie_activation_quantizers:
            return self.quantize_activations_no_range_update(x)
        return self.quantize_activations(x)

    def extra_repr(self):
        return f"tie_activation_quantizers={self.tie_activation_quantizers}"


class Flattener(nn.Module):
    def forward(self, x):
        return x.view(x.shape[0], -1)


def _next_bn(module, i):
    return len(module) > i + 1 and isinstance(module[i + 1], (nn.BatchNorm2d, nn.BatchNorm1d))


def _get_act(module, i):
    """conv + act, or conv + bn + act (replace_operations_with_approx_ops.py:203-217)."""
    acts = tuple(activations_set)
    if len(module) - i > 1 and isinstance(module[i + 1], acts):
        return module[i + 1], i + 1
    if len(module) - i > 2 and _next_bn(module, i) and isinstance(module[i + 2], acts):
        return module[i + 2], i + 2
    return None, None


def _module_args(mod, act):
    if isinstance(mod, _ConvNd):
        kw = dict(in_channels=mod.in_channels, out_channels=mod.out_channels, kernel_size=mod.kernel_size,
                  stride=mod.stride, padding=mod.padding, dilation=mod.dilation, groups=mod.groups,
                  bias=mod.bias is not None)
    elif isinstance(mod, nn.Linear):
        kw = dict(in_features=mod.in_features, out_features=mod.out_features, bias=mod.bias is not None)
    elif isinstance(mod, nn.LayerNorm):  # replace_operations_with_approx_ops.py:240-242
        kw = dict(normalized_shape=mod.normalized_shape, eps=mod.eps)
    else:
        raise ValueError(f"no approx operator for {type(mod).__name__}")
    kw["activation"] = act
    return kw


def _check_on_path(mod):
    if isinstance(mod, _OFF_PATH):
        raise NotImplementedError(f"{type(mod).__name__} maps to a non-approx quantized layer in the reference "
                                  "(autoquant_utils.py); it is outside the approx hot path")


def fold_bn(module, i, **quant_params):
    """Replace module[i] (+ BN + activation) by its approx operator; BN statistics move into
    the operator, which applies them after the product (replace_operations_with_approx_ops.py:263-286)."""
    bn = _next_bn(module, i)
    act, _ = _get_act(module, i)
    modmap = bn_module_map if bn else non_bn_module_map
    if type(module[i]) not in modmap:
        raise NotImplementedError(f"{type(module[i]).__name__} + BatchNorm is outside the approx hot path")
    new = modmap[type(module[i])](**_module_args(module[i], act), **quant_params)
    new.weight.data = module[i].weight.data.clone()
    if bn:
        b = module[i + 1]
        new.gamma.data = b.weight.data.clone()
        new.beta.data = b.bias.data.clone()
        new.running_mean.data = b.running_mean.data.clone()
        new.running_var.data = b.running_var.data.clone()
        if module[i].bias is not None:
            new.running_mean.data -= module[i].bias.data
            warnings.warn("bias in conv/linear before batch normalization")
        new.epsilon = b.eps
    elif module[i].bias is not None:
        new.bias.data = module[i].bias.data.clone()
    return new, i + int(bool(act)) + int(bn) + 1


def quantize_sequential(model, specials=None, tie_activation_quantizers=False, **quant_params):
    """replace_operations_with_approx_ops.py:289-342."""
    specials = specials or {}
    i, out = 0, []
    while i < len(model):
        m = model[i]
        _check_on_path(m)
        if isinstance(m, QuantizedModule):
            out.append(m)
        elif type(m) in non_bn_module_map:
            new, i = fold_bn(model, i, **quant_params)
            out.append(new)
            continue
        elif type(m) in specials:
            out.append(specials[type(m)](m, **quant_params))
        elif isinstance(m, non_param_modules):
            input_quantizer = None
            if out and isinstance(out[-1], QuantizedModule):
                input_quantizer = out[-1].activation_quantizer
            elif out and isinstance(out[-1], nn.Sequential) and isinstance(out[-1][-1], QuantizedModule):
                input_quantizer = out[-1][-1].activation_quantizer
            if input_quantizer and tie_activation_quantizers:
                out.append(QuantizedActivationWrapper(m, tie_activation_quantizers=True,
                                                      input_quantizer=input_quantizer, **quant_params))
            else:
                out.append(QuantizedActivationWrapper(m, **quant_params))
                if tie_activation_quantizers:
                    warnings.warn("Input quantizer not found, so we do not tie quantizers")
        else:
            out.append(quantize_model(m, specials=specials, **quant_params))
        i += 1
    return nn.Sequential(*out)


def quantize_model(model, specials=None, tie_activation_quantizers=False, **quant_params):
    """replace_operations_with_approx_ops.py:345-384."""
    specials = specials or {}
    _check_on_path(model)
    if isinstance(model, nn.Sequential):
        return quantize_sequential(model, specials, tie_activation_quantizers, **quant_params)
    if type(model) in specials:
        return specials[type(model)](model, **quant_params)
    if isinstance(model, non_param_modules):
        return QuantizedActivationWrapper(model, **quant_params)
    if type(model) in non_bn_module_map:
        q = non_bn_module_map[type(model)](**_module_args(model, None), **quant_params)
        q.weight.data = model.weight.data
        if getattr(model, "bias", None) is not None:
            q.bias.data = model.bias.data
        return q
    q = copy.deepcopy(model)
    if isinstance(q, nn.ModuleList):
        for idx, sub in enumerate(q):
            new = quantize_model(sub, specials=specials, **quant_params)
            if new is not None:
                q[idx] = new
    else:
        for name, sub in q._modules.items():
            new = quantize_model(sub, specials=specials, **quant_params)
            if new is not None:
                setattr(q, name, new)
    return q


# ----------------------------------------------------------------------------------- block tails
FUSE_BLOCK = os.environ.get("FP8A_FUSE_BLOCK", "1") != "0"
def fused_block_tail(block, features, x, residual_fn, clamp, in_image=None, next_layer=None, with_image=False):
    """A residual block's tail fused into its last conv's store (fp8a_conv2d_block):
    quantize_activations(clamp(features(x) + residual)) as one launch for the last conv, when that
    conv runs the fused BN store (BNFusedHijacker.block_epilogue_ok) and the block's activation
    quantizer is a per-tensor FPQuantizer in the fixed-range state (or off).  Returns None when the
    block must run unfused.  residual_fn(x) gives the residual (identity or downsample); clamp is
    (lo, hi) or None.  Same result bit for bit as the reference's order (add, clamp, quantize).

    With CHAIN the block's convolutions hand their outputs to each other as word images
    (WordChain): in_image is x's image (emitted by the previous block), next_layer the
    convolution after the block; with_image=True returns (y, the image emitted for next_layer or
    None)."""
    from .quantization.fp8_quantizer import FPQuantizer
    from .quantization.quantization_manager import Qstates
    from .quantization.quantized_folded_bn import BNFusedHijacker
    if not FUSE_BLOCK or len(features) == 0:
        return None
    last = features[-1]
    if not isinstance(last, BNFusedHijacker) or not last.block_epilogue_ok():
        return None
    q = None
    if block._qa():
        mgr = block.activation_quantizer
        q = getattr(mgr, "quantizer", None)
        if getattr(mgr, "state", None) != Qstates.fix_ranges or not isinstance(q, FPQuantizer) \
                or q.maxval.numel() != 1:
            return None
    residual = residual_fn(x)
    lo, hi = clamp if clamp is not None else (0.0, 0.0)
    post = (residual, int(clamp is not None), lo, hi, q)
    layers = list(features)
    if not chain.CHAIN or not all(isinstance(m, BNFusedHijacker) for m in layers):
        h = features[:-1](x) if len(features) > 1 else x
        y = last(h, post=post)
        return (y, None) if with_image else y
    h, img = x, in_image
    for i, m in enumerate(layers):
        ch = chain.WordChain(img, layers[i + 1] if i + 1 < len(layers) else next_layer)
        h = m(h, post=post, chain=ch) if m is last else m(h, chain=ch)
        img = ch.emitted
    return (h, img) if with_image else h


def fused_linear_tail(block, dense, x, residual, dropout=None, gelu=False):
    """block.quantize_activations(dropout(dense(x)) + residual) as one launch of dense's fused
    linear (fp8a_matmul_block), for the ViT blocks (vit_quantized_approx.py:137-156, 256-262):
    same conditions as fused_block_tail (per-tensor FPQuantizer in the fixed-range state, or
    activation quantization off) plus an inactive dropout.  Returns None when the tail must run
    unfused.  Same result bit for bit as the reference's order (product, + bias, + residual,
    quantize).  residual None with gelu: block.quantize_activations(gelu(dense(x))), the MLP's
    first half (vit_quantized_approx.py:117-135; post_act 2 of fp8a_matmul_block)."""
    from .quantization.fp8_quantizer import FPQuantizer
    from .quantization.quantization_manager import Qstates
    if not FUSE_BLOCK or not hasattr(dense, "tail_ok") or not dense.tail_ok():
        return None
    if dropout is not None and dropout.training and dropout.p > 0:
        return None
    q = None
    if block._qa():
        mgr = block.activation_quantizer
        q = getattr(mgr, "quantizer", None)
        if getattr(mgr, "state", None) != Qstates.fix_ranges or not isinstance(q, FPQuantizer) \
                or q.maxval.numel() != 1:
            return None
    if residual is not None:
        if residual.shape[:-1] != x.shape[:-1] or residual.shape[-1] != dense.out_features:
            return None
        if residual.dtype != torch.float32 or not residual.is_contiguous() or residual.data_ptr() % 16:
            return None  # fp8a_matmul_block takes a dense, 16-byte aligned float32 residual
    return dense(x, post=(residual, 2 if gelu else 0, 0.0, 0.0, q))
