"""QuantizationHijacker (reference: quantization/hijacker.py:32-151).

forward() keeps the reference's ordering exactly (hijacker.py:77-115):
  act-quant input -> quantize weights -> [calibration / original_quantize_res: run_forward
  + res_quantizer] -> [qamaa: run_forward] -> [approx: run_forward] -> activation ->
  [output act-quant].  The ValueError for approx/qamaa without res_quantizer_flag is kept.
"""
import copy
import os

from torch import nn

from .base_quantized_classes import QuantizedModule
from .fp8_quantizer import FPQuantizer
from .quantization_manager import QuantizationManager, Qstates
from .range_estimators import CurrentMinMaxEstimator

activations_set = [nn.ReLU, nn.ReLU6, nn.Hardtanh, nn.Sigmoid, nn.Tanh, nn.GELU, nn.PReLU, nn.SiLU, nn.Hardswish,
                   nn.Hardsigmoid]


class QuantizationHijacker(QuantizedModule):
    # fused input quantization (MI355X-side, same result bit for bit): in the fixed-range approx
    # forward the input fake-quant runs inside the approx op (fp8a_conv2d_qin) instead of as its
    # own pass; FP8A_FUSE_QIN=0 or ``fuse_input_quant = False`` keeps the separate pass
    fuse_input_quant = os.environ.get("FP8A_FUSE_QIN", "1") != "0"

    def __init__(self, *args, activation: nn.Module = None, **kwargs):
        super().__init__(*args, **kwargs)
        if activation:
            assert isinstance(activation, tuple(activations_set)), str(activation)
        self.activation_function = copy.deepcopy(activation) if activation else None
        mk = dict(qmethod=self.act_method, init=self.act_range_method, qparams=self.act_qparams,
                  range_estim_params=self.act_range_options)
        self.activation_quantizer = QuantizationManager(**mk)
        self.res_quantizer = QuantizationManager(**mk)
        if self.weight_range_method is CurrentMinMaxEstimator:
            w_init = dict(percentile=self.percentile)
        else:
            w_init = self.weight_range_options
        self.weight_quantizer = QuantizationManager(qmethod=self.method, init=self.weight_range_method,
                                                    per_channel=self.per_channel_weights, qparams=self.weight_qparams,
                                                    range_estim_params=w_init)

    def _check_res_flag(self):
        if (self.quantize_after_mult_and_add or self.approx_flag) and not self.res_quantizer_flag:
            raise ValueError("quantize_after_mult_and_add or approx_flag is set but res_quantizer_flag is not set. "
                             "you need to set res_quantizer_flag to True if you want to use "
                             "quantize_after_mult_and_add or approx_flag")

    def _fused_input_quantizer(self, qa):
        """The input FPQuantizer when its forward can run inside the approx op: the quantized
        input then feeds nothing but the one approx product of a fixed-range eval forward."""
        if not (self.fuse_input_quant and qa and self.quantize_input and self.fix_ranges_flag
                and not self.original_quantize_res and self.approx_flag and self.res_quantizer_flag
                and not self.quantize_after_mult_and_add and getattr(self, "supports_input_quant_fusion", False)):
            return None
        mgr = self.activation_quantizer
        q = getattr(mgr, "quantizer", None)
        if getattr(mgr, "state", None) != Qstates.fix_ranges or not isinstance(q, FPQuantizer) or q.maxval.numel() != 1:
            return None
        return q

    def _core(self, x, offsets=None, epilogue=None, post=None, chain=None):
        """Shared part of QuantizationHijacker.forward and BNFusedHijacker.forward.  epilogue
        (BNFusedHijacker's fused BN + activation) goes to the approx product only; the caller
        guarantees that product is the only one this forward runs."""
        qa = self._qa()
        fq = self._fused_input_quantizer(qa)
        if self.quantize_input and qa and fq is None:
            x = self.activation_quantizer(x)
        weight, bias = self.get_params()
        res = None
        if not self.fix_ranges_flag or self.original_quantize_res:
            res = self.run_forward(x, weight, bias, offsets=offsets)
            if self.quantize_input and qa and self.res_quantizer_flag:
                res = self.res_quantizer(res)
        if self.res_quantizer_flag and self.quantize_after_mult_and_add:
            res = self.run_forward(x, weight, bias)
        if self.res_quantizer_flag and self.approx_flag:
            kw = {}
            if epilogue is not None:
                kw["epilogue"] = epilogue
            if fq is not None:
                kw["qin"] = fq  # x is unquantized; the op quantizes it and sets fq.custom_bias
            if post is not None:
                kw["post"] = post  # a residual block's tail (BNFusedHijacker.forward)
            if chain is not None:
                kw["chain"] = chain  # the word-image hand-off (model_wrap.WordChain)
            res = self.run_forward(x, weight, bias, offsets=offsets, **kw)
        self._check_res_flag()
        if res is None:  # fixed ranges, no approx / qamaa product and original_quantize_res off: the
            # reference then reads an unassigned `res` (hijacker.py:110, quantized_folded_bn.py:66)
            raise UnboundLocalError("local variable 'res' referenced before assignment")
        return res, qa

    def _epilogue(self, res, qa, activation_done=False):
        if self.activation_function is not None and not activation_done:
            res = self.activation_function(res)
        if not self.quantize_input and qa:
            res = self.activation_quantizer(res)
        return res

    def forward(self, x, offsets=None, post=None):
        """post: ``(residual, clamp, lo, hi, output FPQuantizer or None)`` -- a caller's tail
        q(clamp(y + residual)) fused into the approx op's store (only where the operator's
        ``tail_ok()`` holds; the ViT blocks use it)."""
        if post is not None and not (hasattr(self, "tail_ok") and self.tail_ok()):
            raise AssertionError("fused tail requested where the fused store does not run")
        res, qa = self._core(x, offsets, post=post)
        return self._epilogue(res, qa)

    def get_params(self):
        weight, bias = self.get_weight_bias()
        if self._qw():
            weight = self.quantize_weights(weight)
        return weight, bias

    def quantize_weights(self, weights):
        return self.weight_quantizer(weights)

    def get_weights_fp_bias(self):
        return self.weight_quantizer.get_fp_bias()

    def get_acts_fp_bias(self):
        return self.activation_quantizer.get_fp_bias()

    def get_res_fp_bias(self):
        return self.res_quantizer.get_fp_bias()

    def get_weight_bias(self):
        return self.weight, getattr(self, "bias", None)

    def run_forward(self, x, weight, bias, offsets=None):
        raise NotImplementedError()

    def extra_repr(self):
        return f"{super().extra_repr()}-{'input' if self.quantize_input else 'output'}"
