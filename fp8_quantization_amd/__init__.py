"""fp8_quantization_amd -- MI355X-native approx-FP8 matmul/conv engine.

Drop-in for the approx_v9 hot path of revollllt/FP8_quantization: the HIP library
(csrc/fp8approx.hip, C-ABI include/fp8approx.h) carries every product; this package mirrors the
reference's operator / quantizer surface on top of it.
"""
from . import _lib  # noqa: F401
from .approx_ops import (approx_conv2d, approx_matmul, approx_terms, custom_matmul_vectorize,  # noqa: F401
                            float_to_fpany_absint_torch, fp8_fake_quantize, get_error_table_NN, make_flags,
                            qamaa_conv2d, qamaa_matmul, quant_to_fp_any_vectorize_torch)

__version__ = "0.1.0"
