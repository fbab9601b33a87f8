"""MobileNetV2 built from the drop-in approx operators (workload + model-level parity).

The float network has the layer structure of the reference's models/mobilenet_v2.py (the
tonylins MobileNetV2: conv_bn stem, 17 inverted residual blocks with depthwise 3x3 convs,
1x1 head conv, average pool, dropout + linear classifier) and QuantizedMobileNetV2 wraps it
the way models/mobilenet_v2_quantized_approx.py:11-96 does (quantize_sequential with the
InvertedResidual special and tied pooling quantizer, Flattener, quantized classifier).
The depthwise convolutions (one output channel per group) exercise the reference's
tensor-bias semantics.  Pretrained weights need the network, so weights are
random unless a state dict is loaded.
"""
import math
import os

from torch import nn

from .approx_ops import AvgPool2d
from .model_wrap import Flattener, QuantizedModel, fused_block_tail, quantize_model, quantize_sequential
from .quantization.base_quantized_classes import FP32Acts, QuantizedActivation

# t (expansion), c (channels), n (repeats), s (first stride) -- the MobileNetV2 table
_SETTING = ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
            (6, 320, 1, 1))


def _conv_bn_relu6(cin, cout, k, stride, groups=1, relu=True):
    layers = [nn.Conv2d(cin, cout, k, stride, k // 2, groups=groups, bias=False), nn.BatchNorm2d(cout)]
    if relu:
        layers.append(nn.ReLU6(inplace=True))
    return layers


class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        assert stride in (1, 2)
        self.stride = stride
        hidden = round(inp * expand_ratio)
        self.use_res_connect = stride == 1 and inp == oup
        layers = [] if expand_ratio == 1 else _conv_bn_relu6(inp, hidden, 1, 1)
        layers += _conv_bn_relu6(hidden, hidden, 3, stride, groups=hidden)   # depthwise
        layers += _conv_bn_relu6(hidden, oup, 1, 1, relu=False)              # pointwise-linear
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2(nn.Module):
    def __init__(self, n_class=1000, input_size=224, width_mult=1.0, dropout=0.0):
        super().__init__()
        assert input_size % 32 == 0
        cin = int(32 * width_mult)
        self.last_channel = int(1280 * width_mult) if width_mult > 1.0 else 1280
        feats = [nn.Sequential(*_conv_bn_relu6(3, cin, 3, 2))]
        for t, c, n, s in _SETTING:
            cout = int(c * width_mult)
            for i in range(n):
                feats.append(InvertedResidual(cin, cout, s if i == 0 else 1, expand_ratio=t))
                cin = cout
        feats.append(nn.Sequential(*_conv_bn_relu6(cin, self.last_channel, 1, 1)))
        feats.append(AvgPool2d(input_size // 32))  # nn.AvgPool2d on the HIP kernel (approx_ops.py)
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Sequential(nn.Dropout(dropout), nn.Linear(self.last_channel, n_class))
        self._init()

    def _init(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.weight.data.normal_(0, 0.01)
                m.bias.data.zero_()

    def forward(self, x):
        x = self.features(x)
        x = nn.functional.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.classifier(x)


# FP8A_MBV2_XCHAIN=0: the hand-off only inside the residual blocks (the round-5 wiring)
XCHAIN = os.environ.get("FP8A_MBV2_XCHAIN", "1") != "0"


class QuantizedInvertedResidual(QuantizedActivation):
    """mobilenet_v2_quantized_approx.py:11-23: the residual sum is re-quantized."""

    def __init__(self, inv_res_orig, **quant_params):
        super().__init__(**quant_params)
        self.use_res_connect = inv_res_orig.use_res_connect
        self.conv = quantize_sequential(inv_res_orig.conv, **quant_params)

    def forward(self, x):
        return self.forward_chain(x)[0]

    def forward_chain(self, x, in_image=None, next_layer=None):
        """forward, with the word-image hand-off (chain.WordChain) between the block's convolutions
        and to next_layer (the first convolution of the next block; round 6: also for the blocks
        without a residual, and across blocks): in_image is x's word image.  Returns (output, the
        image emitted for next_layer or None).  The same bits as forward without the hand-off."""
        from . import chain
        from .quantization.quantized_folded_bn import BNFusedHijacker
        if not XCHAIN:
            in_image = next_layer = None
        if self.use_res_connect:
            fused = fused_block_tail(self, self.conv, x, lambda t: t, None, in_image=in_image, next_layer=next_layer,
                                     with_image=True)
            if fused is not None:
                return fused
            return self.quantize_activations(x + self.conv(x)), None
        layers = list(self.conv)
        if not XCHAIN or not chain.CHAIN or not all(isinstance(m, BNFusedHijacker) for m in layers):
            return self.conv(x), None
        h, img = x, in_image
        for i, m in enumerate(layers):  # (the chain acts only in each layer's fused store)
            ch = chain.WordChain(img, layers[i + 1] if i + 1 < len(layers) else next_layer)
            h = m(h, chain=ch)
            img = ch.emitted
        return h, img


class QuantizedMobileNetV2(QuantizedModel):
    """mobilenet_v2_quantized_approx.py:26-96 (quant_setup None / "all" / "FP_logits")."""

    def __init__(self, model_fp, input_size=(1, 3, 224, 224), quant_setup=None, **quant_params):
        super().__init__(input_size)
        quantize_input = quant_setup and quant_setup == "LSQ_paper"
        self.features = quantize_sequential(model_fp.features, tie_activation_quantizers=not quantize_input,
                                            specials={InvertedResidual: QuantizedInvertedResidual}, **quant_params)
        self.flattener = Flattener()
        self.classifier = quantize_model(model_fp.classifier, **quant_params)
        if quant_setup == "FP_logits":
            self.classifier[1].activation_quantizer = FP32Acts()
        elif quant_setup is not None and quant_setup != "all":
            raise ValueError("Quantization setup '{}' not supported for MobilenetV2".format(quant_setup))

    def forward(self, x):
        # the features in order, the inverted-residual blocks handing word images to each other
        mods = list(self.features)
        img = None
        for i, m in enumerate(mods):
            if isinstance(m, QuantizedInvertedResidual):
                nxt = mods[i + 1] if i + 1 < len(mods) else None
                x, img = m.forward_chain(x, img, nxt.conv[0] if isinstance(nxt, QuantizedInvertedResidual) else None)
            else:
                x, img = m(x), None
        return self.classifier(self.flattener(x))


def mobilenet_v2_approx(input_size=224, width_mult=1.0, n_class=1000, bn_stats_batches=0, device=None, **cfg):
    from .resnet_workload import approx_qparams, estimate_bn_statistics
    fp = MobileNetV2(n_class=n_class, input_size=input_size, width_mult=width_mult)
    if bn_stats_batches:
        estimate_bn_statistics(fp, bn_stats_batches, input_shape=(3, input_size, input_size), device=device)
    return QuantizedMobileNetV2(fp, input_size=(1, 3, input_size, input_size), **approx_qparams(**cfg))
