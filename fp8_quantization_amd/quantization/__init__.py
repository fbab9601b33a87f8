"""Quantizer / state-machine surface the approx operators sit on.

Restates the behaviour of the reference's quantization package (revollllt/FP8_quantization,
quantization/*.py) that the approx hot path depends on: the FP8 fake quantizer that produces
the operand biases, the range estimators, the QuantizationManager state machine and the
hijacker forward ordering.  The FP8 quantizer arithmetic runs in libfp8approx.so.
"""
from .fp8_quantizer import FPQuantizer, quantize_to_fp8_ste_MM  # noqa: F401
from .range_estimators import (AllMinMaxEstimator, CurrentMinMaxEstimator, RangeEstimators,  # noqa: F401
                               RunningMinMaxEstimator)
from .quantization_manager import QuantizationManager, QuantizerNotInitializedError, Qstates  # noqa: F401
from .base_quantized_classes import FP32Acts, QuantizedActivation, QuantizedModule  # noqa: F401
from .hijacker import QuantizationHijacker, activations_set  # noqa: F401
from .quantized_folded_bn import BNFusedHijacker  # noqa: F401
