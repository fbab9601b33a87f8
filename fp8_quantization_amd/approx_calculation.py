"""Drop-in approx operator classes (reference: approx/approx_calculation.py:551-1023).

QCustomBNConv2dTorch, QCustomLinearTorch and QCustomConv2dTorch keep the reference's
constructor contract (cls(**layer_args, activation=act, **qparams), with qparams carrying
custom_approx_params and run_method) and its ``run_forward(x, weight, bias, offsets=None)``
surface.  The arithmetic is one fused HIP launch per layer instead of the reference's
per-group, per-output-column Python loop (approx_calculation.py:774-799):

  * conv: im2col + approx GEMM + NCHW epilogue (fp8a_conv2d); single-output-channel groups
    (depthwise) keep the reference's tensor-bias semantics (approx_calculation.py:800-809);
  * linear: approx GEMM on x @ weight.t() consumed in place (fp8a_matmul).

The behaviour lives in mixins so the same run_forward can sit on the reference's own
QuantizationHijacker / BNFusedHijacker (see ``bind_operator_classes`` and INTEGRATION.md).
"""
import os

import weakref

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from .approx_ops import (_bias_dev, _res_quant_params, approx_conv2d, approx_matmul, approx_matmul_block, bias_epilogue,
                         dense_conv2d, dense_format, dense_matmul, grouped_conv2d, make_flags, make_flags_v5, qamaa_conv2d,
                         qamaa_matmul)
from .error_tables import get_comp_table_NN_v5, get_error_table_NN
from .quantization.hijacker import QuantizationHijacker
from .quantization.quantization_manager import QuantizationManager
from .quantization.base_quantized_classes import QuantizedActivation, QuantizedModule
from .quantization.hijacker import activations_set
from .quantization.quantized_folded_bn import BNFusedHijacker
from .chain import ChainConsumerMixin

# the non-approx products on the fp8 matrix core (gemm_dense.h); FP8A_DENSE=0: torch's fp32 contraction
DENSE_EXACT = os.environ.get("FP8A_DENSE", "1") != "0"

# (the hijacker bases too: the reference's replace_operations_with_approx_ops takes them from its
# `from approx.approx_calculation import *`, INTEGRATION.md §3 Option A)
__all__ = ["QCustomBNConv2dTorch", "QCustomLinearTorch", "QCustomConv2dTorch", "ApproxOpMixin",
           "ApproxConv2dMixin", "ApproxLinearMixin", "ExactConv2dMixin", "bind_operator_classes",
           "QuantizationHijacker", "BNFusedHijacker", "QuantizationManager",
           "QuantizedActivation", "QuantizedModule", "activations_set"]


class ApproxOpMixin:
    """approx_multiply and its configuration plumbing (approx_calculation.py:749-814, 921-999)."""

    def _approx_config(self):
        p = self.custom_approx_params
        E, M = p["expo_width"], p["mant_width"]
        if p.get("approx_version", 9) == 5:
            # opt-in extension: the v5 integer-adder model with live sim_hw_add_OFUF /
            # with_OF_opt / with_UF_opt (approx_v5.py); without withComp, the zero table the v5
            # harness passes for "no compensation"
            table = get_comp_table_NN_v5(E, M, True, p["dnsmp_factor"], p.get("zero_table_ext", False)) \
                if p["withComp"] else \
                torch.zeros((2 ** M, 2 ** M), dtype=torch.int32)
            return E, M, table, make_flags_v5(p.get("sim_hw_add_OFUF", False), p.get("with_OF_opt", False),
                                              p.get("with_UF_opt", False))
        # get_error_table_NN runs first, as in the reference: unsupported formats raise
        # ValueError even when approx_flag is off (approx_calculation.py:772)
        # (zero_table_ext: the opt-in all-zero table for formats the reference has none for, E5M2)
        table = get_error_table_NN(E, M, withComp=p["withComp"], dnsmp_factor=p["dnsmp_factor"],
                                   zero_table_ext=p.get("zero_table_ext", False))
        flags = make_flags(p["with_approx"], p["with_s2nn2s_opt"], p["quant_btw_mult_accu"], p["golden_clip_OF"])
        return E, M, table, flags

    @staticmethod
    def _default_bias(b, E, device):
        # approx_calculation.py:766-767: a missing act/res bias falls back to 2^(E-1)
        # (a cached device tensor: no host-to-device copy per forward, which a captured graph forbids)
        return b if b is not None else _bias_dev(2 ** (E - 1), device)

    def _qamaa_params(self):
        return _res_quant_params(self.res_quantizer)

    def approx_multiply(self, x, y, x_bias, y_bias, res_bias):
        """x [M, K] @ y [K, N] with the operator's approx configuration."""
        E, M, table, flags = self._approx_config()
        x_bias = self._default_bias(x_bias, E, x.device)
        res_bias = self._default_bias(res_bias, E, x.device)
        if y.shape[1] != 1:
            if self.approx_flag:
                return approx_matmul(x, y, E, M, x_bias, y_bias, res_bias, table, flags=flags)
            if self.quantize_after_mult_and_add:  # approx_calculation.py:787-795
                return qamaa_matmul(x, y, *self._qamaa_params())
            return self._exact_product(x, y, M)
        if self.approx_flag:  # single column: biases stay tensors -> tensor-bias semantics (F5)
            tb = 0 if flags & _lib.V5 else _lib.TB  # (v5 never had tensor-bias semantics)
            return approx_matmul(x, y, E, M, x_bias, y_bias, res_bias, table, flags=flags | tb)
        return self._exact_product(x, y, M)

    def _exact_product(self, x, y, M):
        """The non-approx ``x @ y`` (approx_calculation.py:797, 811): on the GPU the matrix-core
        product (dense_format: the bf16 form, exact for every FP8 / E3M4 / E2M5 grid value) when
        both operands went through this layer's FP8 quantizers, else the fp32 contraction (also
        with FP8A_DENSE=0: A/B measurements).  Unquantized operands would mark every 64 x 64 unit
        of the matrix-core launch for its fp32 recompute (dn_fix), far slower than torch's."""
        fmt = dense_format(M) if DENSE_EXACT and self._operands_quantized() else None
        if x.is_cuda and fmt is not None:
            return dense_matmul(x, y, fmt)
        return x @ y

    def _operands_quantized(self):
        """Weights and activations both FP8-quantized in this forward (quantization on for both;
        the hijacker quantizes the input, or the previous layer's output quantizer did)."""
        if hasattr(self, "_qw") and hasattr(self, "_qa"):
            return bool(self._qw() and self._qa())
        # (the reference's own QuantizedModule, bind_operator_classes: its state buffers)
        qw, qa = getattr(self, "_quant_w", None), getattr(self, "_quant_a", None)
        return qw is not None and qa is not None and bool(qw.reshape(-1)[0]) and bool(qa.reshape(-1)[0])

    def multiply(self, x, y):
        return torch.matmul(x, y)


class ApproxConv2dMixin(ApproxOpMixin, ChainConsumerMixin):
    """run_forward of QCustomBNConv2dTorch (approx_calculation.py:822-917)."""

    def im2col(self, input_data, kernel_height, kernel_width, stride, padding, dilation):
        Bn, C, H, W = input_data.shape
        Ho = (H + 2 * padding[0] - dilation[0] * (kernel_height - 1) - 1) // stride[0] + 1
        Wo = (W + 2 * padding[1] - dilation[1] * (kernel_width - 1) - 1) // stride[1] + 1
        x = input_data.contiguous().float()
        out = torch.empty((Bn * Ho * Wo, C * kernel_height * kernel_width), dtype=torch.float32, device=x.device)
        rc = _lib.load().fp8a_im2col(_lib.dev_ptr(x), _lib.dev_ptr(out), Bn, C, H, W, kernel_height, kernel_width,
                                     stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1],
                                     _lib.stream_ptr(x.device))
        _lib.check(rc, "fp8a_im2col")
        return out

    supports_bn_act_epilogue = True
    supports_input_quant_fusion = True

    def run_forward(self, x, weight, bias, offsets=None, epilogue=None, qin=None, post=None, chain=None):
        """qin: the layer's input FPQuantizer when the hijacker fused it (x unquantized; the op
        applies it and its custom_bias is set as its own forward would).  post: ``(residual,
        clamp, lo, hi, output FPQuantizer or None)`` of a residual block's tail (quantized_folded_bn
        .BNFusedHijacker.forward); the output quantizer's custom_bias is set likewise.  chain: a
        model_wrap.WordChain -- x's word image from the previous convolution (used with qin) and /
        or the next convolution to emit one for (fp8a_conv2d_chain, bit-identical results)."""
        x = x.contiguous()
        weight = weight.contiguous()
        if epilogue is not None and (bias is not None or not self.approx_flag):
            raise AssertionError("the fused BN epilogue needs the approx product without a conv bias")
        if qin is not None and not self.approx_flag:
            raise AssertionError("the fused input quantizer needs the approx product")
        w_bias = self.get_weights_fp_bias()
        a_bias = self.get_acts_fp_bias()
        r_bias = self.get_res_fp_bias()
        E, M, table, flags = self._approx_config()
        if self.approx_flag:
            if w_bias is None:  # the reference indexes weight_fp_bias[...] (approx_calculation.py:868)
                raise TypeError("'NoneType' object is not subscriptable")
            args = dict(flags=flags, stride=self.stride, padding=self.padding, dilation=self.dilation,
                        groups=self.groups, epilogue=epilogue)
            ch = chain.request(self, x, qin) if chain is not None else None
            if ch is not None:
                args["chain"] = ch
            if qin is not None or post is not None or ch is not None:
                qt = lambda q: (q.maxval, q.n_bits, q._mbits_int, q.sign_bits)  # noqa: E731
                pq = None
                if post is not None:
                    pq = post[4]
                    args["post"] = tuple(post[:4]) + ((qt(pq) if pq is not None else None),)
                a_b = None if qin is not None else self._default_bias(a_bias, E, x.device)
                out, ib, ob = approx_conv2d(x.detach(), weight.detach(), E, M, a_b, w_bias,
                                            self._default_bias(r_bias, E, x.device), table,
                                            qin=qt(qin) if qin is not None else None, **args)
                if qin is not None:
                    qin.custom_bias = ib
                if pq is not None:
                    pq.custom_bias = ob
                if ch is not None:
                    chain.done(ch)
            else:
                out = approx_conv2d(x.detach(), weight.detach(), E, M, self._default_bias(a_bias, E, x.device),
                                    w_bias, self._default_bias(r_bias, E, x.device), table, **args)
        elif self.quantize_after_mult_and_add and self.out_channels // self.groups != 1:
            out = qamaa_conv2d(x.detach(), weight.detach(), *self._qamaa_params(), stride=self.stride,
                               padding=self.padding, dilation=self.dilation, groups=self.groups)
        else:  # exact product (also qamaa's single-column groups, approx_calculation.py:810-811)
            out = exact_conv2d(self, x.detach(), weight.detach(), M)
        if bias is not None:
            out += bias.view(1, -1, 1, 1)
        return out


def exact_conv2d(mod, x, w, M):
    """The exact convolution product of ``mod`` (a conv hijacker) on CUDA tensors: grouped /
    depthwise convs on fp8a_grouped_conv2d (the reference's per-group ``x @ y[:, i]``,
    approx_calculation.py:797 / 686-711: fp32 FMAs, any input), groups = 1 on the matrix core
    (dense_conv2d, :811) when both operands went through FP8 quantizers (else the fp32 contraction:
    the bf16 form would send every unit to its fp32 recompute).  CPU tensors, FP8A_DENSE=0 (A/B
    measurements) and wide-mantissa formats: F.conv2d."""
    if x.is_cuda and DENSE_EXACT:
        if mod.groups > 1:
            return grouped_conv2d(x, w, mod.groups, mod.stride, mod.padding, mod.dilation)
        fmt = dense_format(M) if ApproxOpMixin._operands_quantized(mod) else None
        if fmt is not None:
            return dense_conv2d(x, w, fmt, mod.stride, mod.padding, mod.dilation)
    return F.conv2d(x, w, None, mod.stride, mod.padding, mod.dilation, mod.groups)


class ExactConv2dMixin:
    """run_forward of QCustomConv2dTorch: exact fp32 product (approx_calculation.py:660-719), on
    the HIP kernels for CUDA tensors (exact_conv2d)."""

    def run_forward(self, x, weight, bias, offsets=None):
        params = getattr(self, "custom_approx_params", None) or {}
        out = exact_conv2d(self, x.contiguous().detach(), weight.contiguous().detach(), params.get("mant_width", 3))
        if bias is not None:
            out += bias.view(1, -1, 1, 1)
        return out


class ApproxLinearMixin(ApproxOpMixin):
    """run_forward of QCustomLinearTorch (approx_calculation.py:1007-1023).

    Like the reference, only 2-D inputs are accepted (a 3-D [B, T, K] input fails the
    A.shape[1] == B.shape[0] assertion); set ``flatten_leading_dims = True`` on
    the class or instance for the extension that folds leading dims into rows (ViT linears).

    The approx product, the linear's bias and -- in the fixed-range eval forward -- the input
    quantizer (``qin``) and a caller's residual tail (``post``) run as one fp8a_matmul_block
    launch; same values as the reference's separate passes (quantize, product, ``out += bias``,
    add, quantize).  ``fuse_linear_block = False`` (or FP8A_FUSE_LINEAR=0) keeps the separate
    passes.
    """
    flatten_leading_dims = False
    fuse_linear_block = os.environ.get("FP8A_FUSE_LINEAR", "1") != "0"

    @property
    def supports_input_quant_fusion(self):
        return self._block_ok()

    def _block_ok(self):
        # (with autograd recording a trainable bias, the separate `out += bias` keeps its gradient)
        p = self.custom_approx_params
        b = getattr(self, "bias", None)
        return (self.fuse_linear_block and self.approx_flag and self.out_features != 1
                and p.get("approx_version", 9) != 5 and self.get_weights_fp_bias() is not None
                and not (b is not None and b.requires_grad and torch.is_grad_enabled()))

    def tail_ok(self):
        """Whether forward(x, post=...) fuses a caller's residual tail: the fixed-range eval
        forward reduces to this one approx product and nothing follows it inside the layer."""
        return (self._block_ok() and self.fix_ranges_flag and not self.original_quantize_res and not self.training
                and self.res_quantizer_flag and not self.quantize_after_mult_and_add
                and self.activation_function is None and (self.quantize_input or not self._qa()))

    def _bias_epilogue(self, bias, device):
        """{1, bias} store epilogue, rebuilt only when the bias tensor changes."""
        if bias is None:
            return None
        # keyed on the tensor object as well: a replaced bias (new Parameter, load_state_dict with
        # assign=True) may reuse the old storage address with a matching version counter
        key = (bias._version, bias.data_ptr(), device)
        cached = getattr(self, "_bias_epi_cache", None)
        if cached is None or cached[0] != key or cached[1]() is not bias:
            cached = (key, weakref.ref(bias), bias_epilogue(bias, device))
            self._bias_epi_cache = cached
        return cached[2]

    def run_forward(self, x, weight, bias, offsets=None, qin=None, post=None):
        x = x.contiguous()
        weight = weight.contiguous()
        lead = None
        if x.dim() != 2:
            if not self.flatten_leading_dims:
                raise AssertionError(f"approx linear expects a 2-D input, got {tuple(x.shape)} (SURVEY F4)")
            lead = x.shape[:-1]
            x = x.reshape(-1, x.shape[-1])
        if self._block_ok():
            E, M, table, flags = self._approx_config()
            qt = lambda q: (q.maxval, q.n_bits, q._mbits_int, q.sign_bits)  # noqa: E731
            pq, pt = None, None
            if post is not None:
                pq = post[4]
                res = post[0].reshape(-1, weight.shape[0]) if post[0] is not None else None
                pt = (res,) + tuple(post[1:4]) + ((qt(pq) if pq is not None else None),)
            out, ib, ob = approx_matmul_block(
                x.detach(), weight.detach().t(), E, M,
                None if qin is not None else self._default_bias(self.get_acts_fp_bias(), E, x.device),
                self.get_weights_fp_bias(), self._default_bias(self.get_res_fp_bias(), E, x.device), table, flags,
                bias_epi=self._bias_epilogue(bias, x.device), qin=qt(qin) if qin is not None else None, post=pt)
            if qin is not None:
                qin.custom_bias = ib
            if pq is not None:
                pq.custom_bias = ob
        else:
            if qin is not None or post is not None:
                raise AssertionError("fused input quantization / tail without the fused linear launch")
            out = self.approx_multiply(x.detach(), weight.detach().t(), self.get_acts_fp_bias(),
                                       self.get_weights_fp_bias(), self.get_res_fp_bias())
            if bias is not None:
                out += bias
        if lead is not None:
            out = out.reshape(*lead, out.shape[-1])
        return out


def bind_operator_classes(hijacker_cls=QuantizationHijacker, bnfused_cls=BNFusedHijacker):
    """Build the three operator classes on top of any hijacker implementation exposing the
    reference surface (get_*_fp_bias, approx_flag, custom_approx_params, ...)."""
    bn_conv = type("QCustomBNConv2dTorch", (ApproxConv2dMixin, bnfused_cls, nn.Conv2d), {})
    linear = type("QCustomLinearTorch", (ApproxLinearMixin, hijacker_cls, nn.Linear), {})
    conv = type("QCustomConv2dTorch", (ExactConv2dMixin, hijacker_cls, nn.Conv2d), {})
    return bn_conv, linear, conv


class QCustomBNConv2dTorch(ApproxConv2dMixin, BNFusedHijacker, nn.Conv2d):
    pass


class QCustomLinearTorch(ApproxLinearMixin, QuantizationHijacker, nn.Linear):
    pass


class QCustomConv2dTorch(ExactConv2dMixin, QuantizationHijacker, nn.Conv2d):
    pass
