"""Range estimators used by the approx scripts (reference: quantization/range_estimators.py:56-125).

current_minmax (weights, per channel), allminmax (activations, running min/max over every
calibration batch) and running_minmax (EMA).  Plain torch reductions on the device.
"""
from torch import nn


def _minmax(x, per_channel):
    if per_channel:
        flat = x.reshape(x.shape[0], -1)
        return flat.min(-1)[0].detach(), flat.max(-1)[0].detach()
    return x.min().detach(), x.max().detach()


class _Estimator(nn.Module):
    def __init__(self, per_channel=False, quantizer=None, **kwargs):
        super().__init__()
        self.per_channel = per_channel
        self.quantizer = quantizer
        self.current_xmin = None
        self.current_xmax = None

    def reset(self):
        self.current_xmin = self.current_xmax = None


class CurrentMinMaxEstimator(_Estimator):
    def __init__(self, percentile=None, **kwargs):
        super().__init__(**kwargs)
        if percentile:
            raise NotImplementedError("percentile ranges are not used on the approx path")

    def forward(self, x):
        self.current_xmin, self.current_xmax = _minmax(x, self.per_channel)
        return self.current_xmin, self.current_xmax


class AllMinMaxEstimator(_Estimator):
    def forward(self, x):
        lo, hi = _minmax(x, self.per_channel)
        if self.current_xmin is None:
            self.current_xmin, self.current_xmax = lo, hi
        else:
            self.current_xmin = self.current_xmin.minimum(lo)
            self.current_xmax = self.current_xmax.maximum(hi)
        return self.current_xmin, self.current_xmax


class RunningMinMaxEstimator(_Estimator):
    def __init__(self, momentum=0.9, **kwargs):
        super().__init__(**kwargs)
        self.momentum = momentum

    def forward(self, x):
        lo, hi = _minmax(x, self.per_channel)
        if self.current_xmin is None:
            self.current_xmin, self.current_xmax = lo, hi
        else:
            a = self.momentum
            self.current_xmin = (1 - a) * lo + a * self.current_xmin
            self.current_xmax = (1 - a) * hi + a * self.current_xmax
        return self.current_xmin, self.current_xmax


class _Choice:
    def __init__(self, cls):
        self.cls = cls


class RangeEstimators:
    current_minmax = _Choice(CurrentMinMaxEstimator)
    allminmax = _Choice(AllMinMaxEstimator)
    running_minmax = _Choice(RunningMinMaxEstimator)
