"""ResNet-18 / ResNet-50 built from the drop-in approx operators (bench workload).

Mirrors the module structure QuantizedResNet gives torchvision's ResNet in the reference
(models/resnet_quantized_approx.py:11-130 + quantize_model / fold_bn,
approx/replace_operations_with_approx_ops.py:263-384): every conv+BN pair becomes a
QCustomBNConv2dTorch (approx), the fc a QCustomLinearTorch (approx), each residual block
quantizes its output, the average pool re-uses the last block's activation quantizer without
updating its range.  torchvision is not installed and pretrained weights need the network, so
weights are random (kaiming, as torchvision initialises them); shapes are the real ones.
"""
import torch
from torch import nn

from .approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
from .quantization import FPQuantizer, RangeEstimators
from .quantization.base_quantized_classes import QuantizedActivation, QuantizedModule


def approx_qparams(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False, with_approx=True,
                   with_s2nn2s_opt=True, quant_btw_mult_accu=True, golden_clip_OF=False, n_bits=8, run_method=None):
    """qparams exactly as the reference scripts build them (utils/click_options.py:544-606,
    scripts/generated_scripts.py): per-channel current_minmax weights, allminmax activations,
    quantize_input, FP8 quantizer with set_maxval, approx + res_quantizer run method."""
    return dict(
        method=FPQuantizer, act_method=FPQuantizer, n_bits=n_bits, n_bits_act=n_bits, per_channel_weights=True,
        weight_range_method=RangeEstimators.current_minmax.cls, weight_range_options={},
        act_range_method=RangeEstimators.allminmax.cls, act_range_options={}, quantize_input=True,
        fp8_kwargs=dict(maxval=None, mantissa_bits=mant_width, set_maxval=True, learn_maxval=False,
                        learn_mantissa_bits=False, mse_include_mantissa_bits=False, allow_unsigned=False),
        custom_approx_params=dict(expo_width=expo_width, mant_width=mant_width, dnsmp_factor=dnsmp_factor,
                                  withComp=withComp, with_approx=with_approx, with_s2nn2s_opt=with_s2nn2s_opt,
                                  sim_hw_add_OFUF=False, with_OF_opt=False, with_UF_opt=False,
                                  golden_clip_OF=golden_clip_OF, quant_btw_mult_accu=quant_btw_mult_accu,
                                  debug_mode=False, self_check_mode=False),
        run_method=dict(run_method) if run_method else dict(
            approx_flag=True, quantize_after_mult_and_add=False, res_quantizer_flag=True, original_quantize_res=False))


def _conv(qp, cin, cout, k, stride, pad, relu):
    m = QCustomBNConv2dTorch(in_channels=cin, out_channels=cout, kernel_size=k, stride=stride, padding=pad,
                             bias=False, activation=nn.ReLU() if relu else None, **qp)
    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
    return m


class ApproxBlock(QuantizedActivation):
    """QuantizedBlock (models/resnet_quantized_approx.py:11-41) for Basic / Bottleneck blocks."""

    def __init__(self, qp, cin, planes, stride, bottleneck):
        super().__init__(**{k: v for k, v in qp.items() if k not in ("custom_approx_params",)})
        exp = 4 if bottleneck else 1
        if bottleneck:
            feats = [_conv(qp, cin, planes, 1, 1, 0, True), _conv(qp, planes, planes, 3, stride, 1, True),
                     _conv(qp, planes, planes * exp, 1, 1, 0, False)]
        else:
            feats = [_conv(qp, cin, planes, 3, stride, 1, True), _conv(qp, planes, planes, 3, 1, 1, False)]
        self.features = nn.Sequential(*feats)
        self.downsample = _conv(qp, cin, planes * exp, 1, stride, 0, False) if (stride != 1 or cin != planes * exp) \
            else None
        self.relu = nn.ReLU()
        self.out_channels = planes * exp

    def forward(self, x):
        residual = x if self.downsample is None else self.downsample(x)
        out = self.features(x)
        out += residual
        return self.quantize_activations(self.relu(out))


class TiedAvgPool(QuantizedActivation):
    """QuantizedActivationWrapper(avgpool, tie_activation_quantizers=True) (autoquant_utils.py:125-163)."""

    def __init__(self, qp, input_quantizer):
        super().__init__(**{k: v for k, v in qp.items() if k not in ("custom_approx_params",)})
        self.activation_quantizer = input_quantizer
        self.layer = nn.AdaptiveAvgPool2d((1, 1))

    def forward(self, x):
        x = self.layer(x)
        return self.activation_quantizer.quantizer(x) if self._qa() else x


class ApproxResNet(nn.Module):
    def __init__(self, qp, layers=(2, 2, 2, 2), bottleneck=False, num_classes=1000):
        super().__init__()
        feats = [_conv(qp, 3, 64, 7, 2, 3, True), nn.MaxPool2d(3, 2, 1)]
        cin = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            blocks = []
            for b in range(n):
                blk = ApproxBlock(qp, cin, planes, 2 if (b == 0 and i > 0) else 1, bottleneck)
                cin = blk.out_channels
                blocks.append(blk)
            feats.append(nn.Sequential(*blocks))
        self.features = nn.Sequential(*feats)
        self.avgpool = TiedAvgPool(qp, self.features[-1][-1].activation_quantizer)
        self.fc = QCustomLinearTorch(in_features=cin, out_features=num_classes, bias=True, **qp)
        bound = 1.0 / cin ** 0.5
        nn.init.uniform_(self.fc.weight, -bound, bound)
        nn.init.uniform_(self.fc.bias, -bound, bound)

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.fc(x.reshape(x.shape[0], -1))

    # QuantizedModel-style switches (base_quantized_model.py)
    def _each(self, fn):
        for m in self.modules():
            if isinstance(m, QuantizedModule):
                fn(m)

    def quantized(self):
        self._each(lambda m: m.quantized())

    def estimate_ranges(self):
        self._each(lambda m: m.estimate_ranges())

    def fix_ranges(self):
        self._each(lambda m: m.fix_ranges())


def resnet18_approx(**cfg):
    return ApproxResNet(approx_qparams(**cfg), (2, 2, 2, 2), bottleneck=False)


def resnet50_approx(**cfg):
    return ApproxResNet(approx_qparams(**cfg), (3, 4, 6, 3), bottleneck=True)


def approx_layer_shapes(model, image_hw=224):
    """(name, M_per_image, K, N, groups) of every approx product for one image."""
    shapes, hooks = [], []

    def conv_hook(mod, inp, out):
        x = inp[0]
        cog = mod.out_channels // mod.groups
        K = (mod.in_channels // mod.groups) * mod.kernel_size[0] * mod.kernel_size[1]
        shapes.append((type(mod).__name__, out.shape[2] * out.shape[3], K, cog, mod.groups))
        del x

    def lin_hook(mod, inp, out):
        shapes.append((type(mod).__name__, 1, mod.in_features, mod.out_features, 1))

    for m in model.modules():
        if isinstance(m, QCustomBNConv2dTorch):
            hooks.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, QCustomLinearTorch):
            hooks.append(m.register_forward_hook(lin_hook))
    return shapes, hooks


def approx_macs_per_image(shapes):
    return sum(Mi * K * N * g for (_, Mi, K, N, g) in shapes)
