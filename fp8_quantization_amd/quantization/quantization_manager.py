"""QuantizationManager (reference: quantization/quantization_manager.py:89-139).

States: estimate_ranges (every call updates the range estimate, then quantizes),
fix_ranges (quantize only).  get_fp_bias() exposes the quantizer's custom_bias, the bias the
approx operators read (hijacker.py:130-137).  fix_ranges raises QuantizerNotInitializedError
for a quantizer that reports itself uninitialized (quantization_manager.py:93-98); the FP8
quantizer always reports initialized, as the reference's does (fp8_quantizer.py:252-254).
"""
import enum

from torch import nn

from .range_estimators import RangeEstimators


class QuantizerNotInitializedError(Exception):
    """quantization/quantizers/utils.py:6-12."""

    def __init__(self):
        super().__init__("Quantizer has  not been initialized yet")


class Qstates(enum.Enum):
    estimate_ranges = 1
    fix_ranges = 2
    learn_ranges = 3
    estimate_ranges_train = 4


class QuantizationManager(nn.Module):
    def __init__(self, qmethod=None, init=RangeEstimators.current_minmax.cls, per_channel=False, x_min=None,
                 x_max=None, qparams=None, range_estim_params=None):
        super().__init__()
        self.state = Qstates.estimate_ranges
        self.qmethod = qmethod
        self.init = init
        self.per_channel = per_channel
        self.qparams = qparams or {}
        self.range_estim_params = range_estim_params or {}
        self.quantizer = qmethod(per_channel=per_channel, **self.qparams)
        self.quantizer.state = self.state
        self.range_estimator = None
        if x_min is not None and x_max is not None:
            self.set_quant_range(x_min, x_max)
            self.fix_ranges()
        else:
            self.range_estimator = init(per_channel=per_channel, quantizer=self.quantizer, **self.range_estim_params)

    @property
    def n_bits(self):
        return self.quantizer.n_bits

    def _set_state(self, st):
        self.state = st
        self.quantizer.state = st

    def estimate_ranges(self):
        self._set_state(Qstates.estimate_ranges)

    def fix_ranges(self):
        if not self.quantizer.is_initialized:  # quantization_manager.py:93-98
            raise QuantizerNotInitializedError()
        self._set_state(Qstates.fix_ranges)

    def estimate_ranges_train(self):
        self._set_state(Qstates.estimate_ranges_train)

    def learn_ranges(self):
        self.quantizer.make_range_trainable()
        self._set_state(Qstates.learn_ranges)

    def reset_ranges(self):
        self.range_estimator.reset()
        self.quantizer.reset()
        self.estimate_ranges()

    def forward(self, x):
        if self.state == Qstates.estimate_ranges or (self.state == Qstates.estimate_ranges_train and self.training):
            lo, hi = self.range_estimator(x)
            self.set_quant_range(lo, hi)
        return self.quantizer(x)

    def get_fp_bias(self):
        return self.quantizer.custom_bias

    def set_quant_range(self, x_min, x_max):
        self.quantizer.set_quant_range(x_min, x_max)

    def extra_repr(self):
        return f"state={self.state.name}"
