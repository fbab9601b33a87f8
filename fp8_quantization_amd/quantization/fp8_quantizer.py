"""FP8 fake quantizer (reference: quantization/quantizers/fp8_quantizer.py:97-173, 191-319).

quantize_to_fp8_ste_MM keeps its signature and return value (values, float bias); the
per-element arithmetic is the HIP kernel fp8a_fp8_quantize.  FPQuantizer keeps the
reference's attribute surface: n_bits, mantissa_bits (tensor), maxval (tensor), sign_bits,
custom_bias (set by every forward), set_quant_range / fix_ranges.
"""
import torch
from torch import nn

from ..approx_ops import fp8_fake_quantize


def quantize_to_fp8_ste_MM(x_float, n_bits, maxval, num_mantissa_bits, sign_bits):
    M = int(torch.clamp(torch.round(torch.as_tensor(num_mantissa_bits, dtype=torch.float32)), 1,
                        n_bits - sign_bits).item()) if isinstance(num_mantissa_bits, torch.Tensor) else \
        int(min(max(round(float(num_mantissa_bits)), 1), n_bits - sign_bits))
    maxval = torch.as_tensor(maxval, dtype=torch.float32, device=x_float.device)
    per_row = maxval.numel() != 1
    return fp8_fake_quantize(x_float, maxval, n_bits, M, sign_bits=sign_bits, per_row=per_row)


class FPQuantizer(nn.Module):
    """8-bit floating-point quantizer with a learnable-free custom exponent bias."""

    def __init__(self, n_bits=8, per_channel=False, scale_domain=None, mantissa_bits=4, maxval=3,
                 set_maxval=False, learn_maxval=False, learn_mantissa_bits=False, mse_include_mantissa_bits=True,
                 allow_unsigned=False, **kwargs):
        super().__init__()
        self.n_bits = n_bits
        self.per_channel = per_channel
        self.state = None
        self.ebits = n_bits - mantissa_bits - 1
        self.default_bias = 2 ** (self.ebits - 1)
        default_maxval = (2 - 2 ** (-mantissa_bits)) * 2 ** (2 ** self.ebits - 1 - self.default_bias)
        self.maxval = torch.Tensor([maxval if maxval is not None else default_maxval])
        self.mantissa_bits = torch.Tensor([float(mantissa_bits)])
        self._mbits_int = int(mantissa_bits)
        self.set_maxval = set_maxval
        self.learning_maxval = learn_maxval
        self.learning_mantissa_bits = learn_mantissa_bits
        self.mse_include_mantissa_bits = mse_include_mantissa_bits
        self.allow_unsigned = allow_unsigned
        self.sign_bits = 1
        self.custom_bias = None

    @property
    def is_initialized(self):
        # always True, as the reference's FPQuantizer (fp8_quantizer.py:252-254): it starts from a
        # default maxval, so fix_ranges never raises for it (QuantizationManager.fix_ranges)
        return True

    def forward(self, x_float):
        if self.maxval.device != x_float.device:
            self.maxval = self.maxval.to(x_float.device)
        res, self.custom_bias = quantize_to_fp8_ste_MM(x_float, self.n_bits, self.maxval, self._mbits_int,
                                                       self.sign_bits)
        return res

    def set_quant_range(self, x_min, x_max):
        if self.allow_unsigned and bool(torch.all(torch.as_tensor(x_min) >= 0)):
            self.sign_bits = 0
        if self.set_maxval:
            if not isinstance(x_max, torch.Tensor):
                x_max = torch.tensor([float(x_max)], device=self.maxval.device)
                x_min = torch.tensor([float(x_min)], device=self.maxval.device)
            mx = torch.abs(torch.max(torch.abs(x_min), x_max))
            self.maxval = mx.reshape(1) if mx.dim() == 0 else mx

    def fix_ranges(self):
        pass

    def make_range_trainable(self):
        raise NotImplementedError("learned FP8 ranges are outside the approx hot path")

    def reset(self):
        pass

    def extra_repr(self):
        return f"n_bits={self.n_bits}, mantissa_bits={self._mbits_int}, per_channel={self.per_channel}"
