"""BNFusedHijacker (reference: quantization/quantized_folded_bn.py:15-95).

Same state machine as QuantizationHijacker, then F.batch_norm with the layer's own running
statistics (BN is applied after the approx product, not folded into the weights).

Fused epilogue (MI355X-side, same result within fp32 rounding): when the forward reduces to one
approx product followed by eval-mode batch norm -- eval mode, fixed ranges, approx_flag +
res_quantizer_flag, no original_quantize_res / qamaa -- the batch norm and a clamp activation
(ReLU / ReLU6 / Hardtanh) run inside the conv kernel's store instead of as two more passes over
the output (fp8a_conv2d_bn_act).  ``fuse_bn_act = False`` on the class or instance, or
FP8A_FUSE_BN=0 in the environment, keeps the unfused sequence.

Config-1 form (round 4): with approx_flag off and original_quantize_res (BASELINE config 1's
PTQ run) the whole layer -- input quantizer, exact product, res quantizer, eval batch norm, clamp,
output quantizer -- runs as one fused exact convolution (fp8a_dense_conv2d_fused), leaving each
quantizer the custom_bias its own forward would.
"""
import os

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.modules.conv import _ConvNd

from .hijacker import QuantizationHijacker


class BNFusedHijacker(QuantizationHijacker):
    fuse_bn_act = os.environ.get("FP8A_FUSE_BN", "1") != "0"

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

    def _fused_epilogue(self):
        """(scale_shift, act, lo, hi) for the kernel epilogue, or None when the forward is not
        the single-product eval form (see module doc) or the activation is not a clamp."""
        if (not self.fuse_bn_act or self.training or not self.fix_ranges_flag or self.original_quantize_res
                or self.quantize_after_mult_and_add or not self.approx_flag or not self.res_quantizer_flag
                or not getattr(self, "supports_bn_act_epilogue", False)):
            return None
        return self._epilogue_params()

    def _per_tensor_fp8(self, mgr):
        """The FPQuantizer behind a fixed-range QuantizationManager with one maxval, else None."""
        from .fp8_quantizer import FPQuantizer
        from .quantization_manager import Qstates
        q = getattr(mgr, "quantizer", None)
        if getattr(mgr, "state", None) != Qstates.fix_ranges or not isinstance(q, FPQuantizer) or q.maxval.numel() != 1:
            return None
        return q

    def _config1_fused(self, x):
        """The plan of BASELINE config 1's layer (approx_flag off, original_quantize_res, eval, fixed
        ranges) as one fused exact convolution (approx_ops.dense_conv2d_fused): (qin, rq, oq
        FPQuantizers or None, bn epilogue, dense format), or None when the forward is not that form
        (then the unfused sequence below runs)."""
        if (not self.fuse_bn_act or self.training or not self.fix_ranges_flag or not self.original_quantize_res
                or self.approx_flag or self.quantize_after_mult_and_add or not isinstance(self, _ConvNd)
                or not getattr(self, "supports_bn_act_epilogue", False) or not x.is_cuda):
            return None
        from .. import approx_calculation as ac
        from ..approx_ops import dense_format
        if not ac.DENSE_EXACT or not (self._qw() and self._qa()):
            return None
        fmt = dense_format(self._approx_config()[1])
        ep = self._epilogue_params()
        if fmt is None or ep is None:
            return None
        aq = self._per_tensor_fp8(self.activation_quantizer)
        if aq is None:
            return None
        qin = aq if self.quantize_input else None
        rq = None
        if self.quantize_input and self.res_quantizer_flag:
            rq = self._per_tensor_fp8(self.res_quantizer)
            if rq is None:
                return None
        oq = aq if not self.quantize_input else None
        return qin, rq, oq, ep, fmt

    def _epilogue_params(self):
        from ..approx_ops import bn_act_epilogue
        ts = (self.running_mean, self.running_var, self.gamma, self.beta)
        key = tuple((t._version, t.data_ptr(), t.device) for t in ts) + (self.epsilon, id(self.activation_function))
        cached = getattr(self, "_bn_act_cache", None)
        if cached is None or cached[0] != key:
            cached = (key, bn_act_epilogue(*ts, self.epsilon, self.activation_function))
            self._bn_act_cache = cached
        return cached[1]

    def _forward_config1_fused(self, x, plan):
        from ..approx_ops import dense_conv2d_fused
        qin, rq, oq, ep, fmt = plan
        qt = lambda q: None if q is None else (q.maxval, q.n_bits, q._mbits_int, q.sign_bits)  # noqa: E731
        wq = self._fused_weight_quantizer()
        if wq is None:  # get_params' weight quantizer as its own pass
            weight, _ = self.get_params()
        else:  # ... or inside the product's weight loads (the same values, hijacker.py:113-120)
            weight, _ = self.get_weight_bias()
        self._check_res_flag()
        y, b = dense_conv2d_fused(x.detach(), weight.detach(), self.groups, self.stride, self.padding, self.dilation,
                                  fmt, qin=qt(qin), rq=qt(rq), bn=ep, oq=qt(oq), wq=qt(wq))
        for name, q in (("qin", qin), ("rq", rq), ("oq", oq), ("wq", wq)):
            if q is not None:
                q.custom_bias = b[name]  # what the quantizer's own forward leaves (fp8_quantizer.py)
        return y

    def _fused_weight_quantizer(self):
        """The weight FPQuantizer when the fused product can apply it to the weights as it loads
        them: weights quantized (_qw), fixed ranges (so its forward is the bare quantizer,
        quantization_manager.py), one maxval per tensor or per output channel; else None."""
        if not self._qw():
            return None
        from .fp8_quantizer import FPQuantizer
        from .quantization_manager import Qstates
        mgr = self.weight_quantizer
        q = getattr(mgr, "quantizer", None)
        if getattr(mgr, "state", None) != Qstates.fix_ranges or not isinstance(q, FPQuantizer):
            return None
        if q.maxval.numel() not in (1, self.out_channels) or q.maxval.device != self.weight.device:
            return None
        return q

    def _own_output_quantizer(self):
        """This layer's activation FPQuantizer when it quantizes its OUTPUT (quantize_input off,
        fixed ranges, per tensor) and the fused store can apply it (ungrouped, more than one
        output channel per group -- the block tail's store), else None."""
        if self.quantize_input or not self._qa() or self.out_channels // self.groups == 1:
            return None
        return self._per_tensor_fp8(self.activation_quantizer)

    def block_epilogue_ok(self):
        """Whether forward(x, post=...) can fuse a residual block's tail: the fused BN / activation
        store runs, the product is not a tensor-bias (single-output-channel) one, and nothing
        follows the product inside this layer (no output quantizer of its own)."""
        return (self._fused_epilogue() is not None and self.out_channels // self.groups != 1
                and (self.quantize_input or not self._qa()))

    def forward(self, x, post=None, chain=None):
        """post: ``(residual, clamp, lo, hi, output FPQuantizer or None)`` -- the caller's block
        tail y = q(clamp(y + residual)) fused into the store (only when block_epilogue_ok()).
        chain: a model_wrap.WordChain (the word-image hand-off between consecutive convolutions);
        it only acts in the fused store, and records there whether the next image was emitted."""
        if post is None:
            plan = self._config1_fused(x)
            if plan is not None:
                return self._forward_config1_fused(x, plan)
        ep = self._fused_epilogue()
        if post is not None and not self.block_epilogue_ok():
            raise AssertionError("block epilogue requested where the fused store does not run")
        if ep is not None:
            own = self._own_output_quantizer() if post is None else None
            if own is not None:
                # the layer's own output quantizer (quantize_input off) in the store as well: the
                # fused tail with no residual and no clamp, same fq_apply as its own forward
                res, _ = self._core(x, epilogue=ep, post=(None, 0, 0.0, 0.0, own), chain=chain)
                return res
            res, qa = self._core(x, epilogue=ep, post=post, chain=chain)
            return self._epilogue(res, qa, activation_done=True)
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
