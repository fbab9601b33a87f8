#!/usr/bin/env python
"""Drop-in check against the reference's own model wrappers (TEST INFRASTRUCTURE ONLY; run by
tests/test_ref_dropin_cpu.py in a subprocess, in the build container where the reference checkout
is mounted at /root/reference).

Builds the reference's QuantizedMobileNetV2 (models/mobilenet_v2_quantized_approx.py, unmodified,
over its float MobileNetV2: width 0.25, 32x32, 10 classes) through INTEGRATION.md §3's two routes:
  A  -- ``sys.modules["approx.approx_calculation"]`` aliased to this repo's module before the
        reference's replace_operations_with_approx_ops is imported (this repo's quantization
        surface under the reference's wrapper);
  B  -- the reference's own hijackers, with this repo's run_forward mixins bound onto them
        (bind_operator_classes) and the replacement maps pointed at the bound classes.
Prints one JSON object: per approx layer its class and whether it carries this repo's operator
mixin, and the state-dict keys and shapes.  The same import shim as tests/golden/gen_golden.py
(module-level ``device='cuda'`` tensors to the CPU, stub modules for the un-installed cupy /
timm); no forward runs (the operators need the GPU).
"""
import contextlib
import io
import json
import os
import sys
import types

import torch
import torch.nn as nn

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _install_shim():
    orig_tensor, orig_zeros = torch.tensor, torch.zeros

    def _cpu(kw):
        d = kw.get("device")
        if d is not None and str(d).startswith("cuda"):
            kw["device"] = "cpu"
        return kw

    torch.tensor = lambda *a, **kw: orig_tensor(*a, **_cpu(kw))
    torch.zeros = lambda *a, **kw: orig_zeros(*a, **_cpu(kw))
    sys.modules.setdefault("cupy", types.ModuleType("cupy"))
    for m in ("timm", "timm.models", "timm.models.layers", "timm.models.layers.activations",
              "timm.models.layers.activations_me"):
        sys.modules.setdefault(m, types.ModuleType(m))
    for c in ("Swish", "HardSwish", "HardSigmoid"):
        setattr(sys.modules["timm.models.layers.activations"], c, type(c, (nn.Module,), {}))
    for c in ("SwishMe", "HardSwishMe", "HardSigmoidMe"):
        setattr(sys.modules["timm.models.layers.activations_me"], c, type(c, (nn.Module,), {}))
    sys.path.insert(0, REF)
    sys.path.insert(0, ROOT)
    # models/__init__.py imports every wrapper (some need torchvision, absent): the package
    # without its __init__
    pkg = types.ModuleType("models")
    pkg.__path__ = [os.path.join(REF, "models")]
    sys.modules["models"] = pkg


def main(route):
    _install_shim()
    import fp8_quantization_amd.approx_calculation as amd
    if route == "A":
        sys.modules["approx.approx_calculation"] = amd
        from fp8_quantization_amd.resnet_workload import approx_qparams
        qp = approx_qparams(expo_width=4, mant_width=3, dnsmp_factor=3)
    else:
        from quantization.hijacker import QuantizationHijacker
        from quantization.quantized_folded_bn import BNFusedHijacker
        from quantization.quantizers.fp8_quantizer import FPQuantizer
        from quantization.range_estimators import RangeEstimators
        bn_conv, linear, conv = amd.bind_operator_classes(QuantizationHijacker, BNFusedHijacker)
        import approx.replace_operations_with_approx_ops as rep
        rep.bn_module_map[nn.Conv2d] = bn_conv
        rep.non_bn_module_map[nn.Conv2d] = conv
        rep.non_bn_module_map[nn.Linear] = linear
        rep.QCustomBNConv2dTorch = bn_conv  # the name the model wrapper imports from rep
        qp = dict(method=FPQuantizer, act_method=FPQuantizer, n_bits=8, n_bits_act=8, per_channel_weights=True,
                  weight_range_method=RangeEstimators.current_minmax.cls, weight_range_options={},
                  act_range_method=RangeEstimators.allminmax.cls, act_range_options={}, quantize_input=True,
                  fp8_kwargs=dict(maxval=None, mantissa_bits=3, set_maxval=True, learn_maxval=False,
                                  learn_mantissa_bits=False, mse_include_mantissa_bits=False, allow_unsigned=False),
                  custom_approx_params=dict(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False,
                                            with_approx=True, with_s2nn2s_opt=True, sim_hw_add_OFUF=False,
                                            with_OF_opt=False, with_UF_opt=False, golden_clip_OF=False,
                                            quant_btw_mult_accu=True, debug_mode=False, self_check_mode=False),
                  run_method=dict(approx_flag=True, quantize_after_mult_and_add=False, res_quantizer_flag=True,
                                  original_quantize_res=False))
    from models.mobilenet_v2 import MobileNetV2
    from models.mobilenet_v2_quantized_approx import QuantizedMobileNetV2
    torch.manual_seed(88)
    fp = MobileNetV2(n_class=10, input_size=32, width_mult=0.25)
    with contextlib.redirect_stdout(io.StringIO()):
        model = QuantizedMobileNetV2(fp, input_size=(1, 3, 32, 32), **qp)
    layers = {}
    for name, m in model.named_modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            layers[name] = dict(cls=type(m).__name__, module=type(m).__module__,
                                conv_mixin=isinstance(m, amd.ApproxConv2dMixin),
                                linear_mixin=isinstance(m, amd.ApproxLinearMixin),
                                groups=getattr(m, "groups", None))
    state = {k: list(v.shape) for k, v in model.state_dict().items()}
    print(json.dumps(dict(route=route, layers=layers, state=state)))


if __name__ == "__main__":
    main(sys.argv[1])
