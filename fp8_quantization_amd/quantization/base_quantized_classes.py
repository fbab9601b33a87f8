"""QuantizedModule / QuantizedActivation (reference: quantization/base_quantized_classes.py:49-214).

QuantizedModule pops the approx configuration (custom_approx_params, run_method) from the
constructor kwargs exactly like the reference (:76-82) and carries the quantization on/off
switches (_quant_w / _quant_a buffers) and the fix_ranges flag the hijacker forward reads.
"""
import torch
from torch import nn

from .fp8_quantizer import FPQuantizer
from .quantization_manager import QuantizationManager
from .range_estimators import CurrentMinMaxEstimator, RunningMinMaxEstimator


def _set_layer_fix_ranges(layer):
    # (base_quantized_classes.py:23-28: a model-wide fix skips managers whose quantizer is not
    # initialized; QuantizationManager.fix_ranges on one raises QuantizerNotInitializedError)
    if isinstance(layer, QuantizationManager) and layer.quantizer.is_initialized:
        layer.fix_ranges()
    if isinstance(layer, QuantizedModule):
        layer.fix_ranges_flag = True


def _set_layer_estimate_ranges(layer):
    if isinstance(layer, QuantizationManager):
        layer.estimate_ranges()
    if isinstance(layer, QuantizedModule):
        layer.fix_ranges_flag = False


def _set_layer_approx_calculation(layer):
    if isinstance(layer, QuantizedModule) and layer.approx_flag is not None:
        layer.approx_flag = True


_DEFAULT_RUN_METHOD = dict(approx_flag=False, quantize_after_mult_and_add=False, res_quantizer_flag=False,
                           original_quantize_res=False)


class QuantizedModule(nn.Module):
    def __init__(self, *args, method=FPQuantizer, act_method=None, weight_range_method=CurrentMinMaxEstimator,
                 act_range_method=RunningMinMaxEstimator, n_bits=8, n_bits_act=None, per_channel_weights=False,
                 percentile=None, weight_range_options=None, act_range_options=None, scale_domain="linear",
                 act_quant_kwargs=None, weight_quant_kwargs=None, quantize_input=False, fp8_kwargs=None, **kwargs):
        kwargs.pop("act_quant_dict", None)
        self.custom_approx_params = kwargs.pop("custom_approx_params", None)
        self.run_method = kwargs.pop("run_method", None) or dict(_DEFAULT_RUN_METHOD)
        self.approx_flag = self.run_method["approx_flag"]
        self.quantize_after_mult_and_add = self.run_method["quantize_after_mult_and_add"]
        self.res_quantizer_flag = self.run_method["res_quantizer_flag"]
        self.original_quantize_res = self.run_method["original_quantize_res"]
        super().__init__(*args, **kwargs)
        self.method = method
        self.act_method = act_method or method
        self.n_bits = n_bits
        self.n_bits_act = n_bits_act or n_bits
        self.per_channel_weights = per_channel_weights
        self.percentile = percentile
        self.weight_range_method = weight_range_method
        self.weight_range_options = weight_range_options or {}
        self.act_range_method = act_range_method
        self.act_range_options = act_range_options or {}
        self.scale_domain = scale_domain
        self.quantize_input = quantize_input
        self.fp8_kwargs = fp8_kwargs or {}
        self.register_buffer("_quant_w", torch.BoolTensor([False]))
        self.register_buffer("_quant_a", torch.BoolTensor([False]))
        self.act_qparams = dict(n_bits=self.n_bits_act, scale_domain=scale_domain, **(act_quant_kwargs or {}),
                                **self.fp8_kwargs)
        self.weight_qparams = dict(n_bits=self.n_bits, scale_domain=scale_domain, **(weight_quant_kwargs or {}),
                                   **self.fp8_kwargs)
        self.fix_ranges_flag = False

    # quantization switches (host-side bools: no device round trip per forward)
    def quantized_weights(self):
        self._quant_w = torch.BoolTensor([True])

    def full_precision_weights(self):
        self._quant_w = torch.BoolTensor([False])

    def quantized_acts(self):
        self._quant_a = torch.BoolTensor([True])

    def full_precision_acts(self):
        self._quant_a = torch.BoolTensor([False])

    def quantized(self):
        self.quantized_weights()
        self.quantized_acts()

    def full_precision(self):
        self.full_precision_weights()
        self.full_precision_acts()

    def _qw(self):
        return bool(self._quant_w.cpu()[0]) if self._quant_w.device.type != "cpu" else bool(self._quant_w[0])

    def _qa(self):
        return bool(self._quant_a.cpu()[0]) if self._quant_a.device.type != "cpu" else bool(self._quant_a[0])

    def fix_ranges(self):
        self.apply(_set_layer_fix_ranges)
        self.fix_ranges_flag = True

    def estimate_ranges(self):
        self.apply(_set_layer_estimate_ranges)
        self.fix_ranges_flag = False

    def approx_calculation(self):
        self.approx_flag = True
        self.apply(_set_layer_approx_calculation)

    def _apply(self, fn, *args, **kwargs):
        # keep the on/off switches on the host so forward never syncs on them
        qw, qa = self._quant_w, self._quant_a
        out = super()._apply(fn, *args, **kwargs)
        self._quant_w, self._quant_a = qw, qa
        return out


class QuantizedActivation(QuantizedModule):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.activation_quantizer = QuantizationManager(qmethod=self.act_method, qparams=self.act_qparams,
                                                        init=self.act_range_method,
                                                        range_estim_params=self.act_range_options)

    def quantize_activations(self, x):
        return self.activation_quantizer(x) if self._qa() else x

    def forward(self, x):
        return self.quantize_activations(x)


class FP32Acts(nn.Module):
    def forward(self, x):
        return x

    def reset_ranges(self):
        pass
