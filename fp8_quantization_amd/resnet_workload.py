"""ResNet-18 / ResNet-50 built from the drop-in approx operators (bench workload).

The float network has torchvision's ResNet layout and parameter names (conv1 / bn1 / relu /
maxpool / layer1-4 of BasicBlock or Bottleneck / avgpool / fc, so a torchvision checkpoint
loads with ``load_float_weights``), and QuantizedResNet wraps it exactly the way the
reference's models/resnet_quantized_approx.py:11-130 does: the stem and every block's
conv+BN(+ReLU) become QCustomBNConv2dTorch through ``quantize_model`` (fold_bn), each block
re-quantizes its output (QuantizedBlock), the average pool re-uses the last block's quantizer
without updating its range, and the fc is a QCustomLinearTorch.  The quantized model's
state_dict therefore has the reference's keys.  torchvision is not installed and pretrained
weights need the network, so by default weights are random (torchvision's initialisation).
"""
import torch
from torch import nn

from .approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
from .approx_ops import MaxPool2d
from .model_wrap import Flattener, QuantizedActivationWrapper, QuantizedModel, fused_block_tail, quantize_model
from .quantization import FPQuantizer, RangeEstimators
from .quantization.base_quantized_classes import FP32Acts, QuantizedActivation


def approx_qparams(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False, with_approx=True,
                   with_s2nn2s_opt=True, quant_btw_mult_accu=True, golden_clip_OF=False, n_bits=8, run_method=None,
                   zero_table_ext=None, approx_version=9, sim_hw_add_OFUF=False, with_OF_opt=False,
                   with_UF_opt=False):
    """qparams exactly as the reference scripts build them (utils/click_options.py:544-606,
    scripts/generated_scripts.py): per-channel current_minmax weights, allminmax activations,
    quantize_input, FP8 quantizer with set_maxval, approx + res_quantizer run method.

    Extensions (not in the reference): zero_table_ext (None = on exactly for formats the
    reference has no error table for, E5M2: error_tables.get_error_table_NN) and approx_version 5
    (the v5 integer-adder model with live sim_hw_add_OFUF / with_OF_opt / with_UF_opt)."""
    if zero_table_ext is None:
        zero_table_ext = (expo_width, mant_width) not in ((4, 3), (3, 4), (2, 5))
    return dict(
        method=FPQuantizer, act_method=FPQuantizer, n_bits=n_bits, n_bits_act=n_bits, per_channel_weights=True,
        weight_range_method=RangeEstimators.current_minmax.cls, weight_range_options={},
        act_range_method=RangeEstimators.allminmax.cls, act_range_options={}, quantize_input=True,
        fp8_kwargs=dict(maxval=None, mantissa_bits=mant_width, set_maxval=True, learn_maxval=False,
                        learn_mantissa_bits=False, mse_include_mantissa_bits=False, allow_unsigned=False),
        custom_approx_params=dict(expo_width=expo_width, mant_width=mant_width, dnsmp_factor=dnsmp_factor,
                                  withComp=withComp, with_approx=with_approx, with_s2nn2s_opt=with_s2nn2s_opt,
                                  sim_hw_add_OFUF=sim_hw_add_OFUF, with_OF_opt=with_OF_opt, with_UF_opt=with_UF_opt,
                                  golden_clip_OF=golden_clip_OF, quant_btw_mult_accu=quant_btw_mult_accu,
                                  debug_mode=False, self_check_mode=False,
                                  **({"zero_table_ext": True} if zero_table_ext else {}),
                                  **({"approx_version": 5} if approx_version == 5 else {})),
        run_method=dict(run_method) if run_method else dict(
            approx_flag=True, quantize_after_mult_and_add=False, res_quantizer_flag=True, original_quantize_res=False))


def _conv(qp, cin, cout, k, stride, pad, relu):
    """One stand-alone approx conv + BN (+ ReLU) operator (tests)."""
    m = QCustomBNConv2dTorch(in_channels=cin, out_channels=cout, kernel_size=k, stride=stride, padding=pad,
                             bias=False, activation=nn.ReLU() if relu else None, **qp)
    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
    return m


# ------------------------------------------------------------------------- float ResNet (torchvision layout)
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        return self.relu(self.bn2(self.conv2(out)) + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        return self.relu(self.bn3(self.conv3(out)) + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._layer(block, 64, layers[0], 1)
        self.layer2 = self._layer(block, 128, layers[1], 2)
        self.layer3 = self._layer(block, 256, layers[2], 2)
        self.layer4 = self._layer(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _layer(self, block, planes, n, stride):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        blocks = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        blocks += [block(self.inplanes, planes) for _ in range(1, n)]
        return nn.Sequential(*blocks)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def estimate_bn_statistics(model_fp, batches=4, batch_size=32, input_shape=(3, 224, 224), device=None, seed=0):
    """Give a random-init float model trained-like activation ranges: BN running statistics
    become the cumulative mean / variance of its own activations on synthetic ImageNet-normalised
    inputs (what BN statistics are after training).  Without this, eval-mode BN with the
    default (0, 1) statistics lets activations shrink geometrically through a random network
    (MobileNetV2: ~2^-40 by the head), far from any trained model's FP8 ranges."""
    dev = device or next(model_fp.parameters()).device
    model_fp.to(dev)
    bns = [m for m in model_fp.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
    for m in bns:
        m.reset_running_stats()
        m.momentum = None  # cumulative average
    model_fp.train()
    g = torch.Generator(device="cpu").manual_seed(seed)
    with torch.no_grad():
        for _ in range(batches):
            model_fp(torch.randn((batch_size,) + tuple(input_shape), generator=g).to(dev))
    model_fp.eval()
    for m in bns:
        m.momentum = 0.1
    return model_fp


def load_float_weights(model_fp, path):
    """Load a torchvision-format float checkpoint (state dict) without executing pickled code."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model_fp.load_state_dict(sd.get("state_dict", sd) if isinstance(sd, dict) else sd)
    return model_fp


# ------------------------------------------------------------------------- quantized wrappers
class QuantizedBlock(QuantizedActivation):
    """resnet_quantized_approx.py:11-41."""

    def __init__(self, block, **quant_params):
        super().__init__(**quant_params)
        if isinstance(block, Bottleneck):
            feats = nn.Sequential(block.conv1, block.bn1, block.relu, block.conv2, block.bn2, block.relu, block.conv3,
                                  block.bn3)
        else:
            feats = nn.Sequential(block.conv1, block.bn1, block.relu, block.conv2, block.bn2)
        self.features = quantize_model(feats, **quant_params)
        self.downsample = quantize_model(block.downsample, **quant_params) if block.downsample else None
        self.relu = block.relu

    def forward(self, x):
        return self.forward_chain(x)[0]

    def forward_chain(self, x, in_image=None, next_layer=None):
        """forward, with the word-image hand-off (chain.WordChain) in the fused state: in_image is
        x's word image (emitted by the previous block), next_layer the convolution after this
        block.  Returns (output, the image emitted for next_layer or None)."""
        fused = fused_block_tail(self, self.features, x,
                                 lambda t: t if self.downsample is None else self.downsample(t), (0.0, float("inf")),
                                 in_image=in_image, next_layer=next_layer, with_image=True)
        if fused is not None:
            return fused
        residual = x if self.downsample is None else self.downsample(x)
        out = self.features(x)
        out += residual
        return self.quantize_activations(self.relu(out)), None


class QuantizedResNet(QuantizedModel):
    """resnet_quantized_approx.py:44-130 (quant_setup None / "all" / "FP_logits")."""

    def __init__(self, resnet, input_size=(1, 3, 224, 224), quant_setup=None, **quant_params):
        super().__init__(input_size)
        specials = {BasicBlock: QuantizedBlock, Bottleneck: QuantizedBlock}
        feats = nn.Sequential(resnet.conv1, resnet.bn1, resnet.relu, MaxPool2d.from_module(resnet.maxpool),
                              resnet.layer1, resnet.layer2, resnet.layer3, resnet.layer4)
        self.features = quantize_model(feats, specials=specials, **quant_params)
        self.avgpool = QuantizedActivationWrapper(resnet.avgpool, tie_activation_quantizers=True,
                                                  input_quantizer=self.features[-1][-1].activation_quantizer,
                                                  **quant_params)
        self.flattener = Flattener()
        self.fc = quantize_model(resnet.fc, **quant_params)
        if quant_setup == "FP_logits":
            self.fc.activation_quantizer = FP32Acts()
        elif quant_setup is not None and quant_setup != "all":
            raise ValueError("Quantization setup '{}' not supported for Resnet".format(quant_setup))

    def forward(self, x):
        # the features in order, the blocks handing word images to each other (chain.WordChain)
        mods = [b for m in self.features for b in (m if isinstance(m, nn.Sequential) else [m])]
        img = None
        for i, m in enumerate(mods):
            if isinstance(m, QuantizedBlock):
                nxt = mods[i + 1] if i + 1 < len(mods) else None
                x, img = m.forward_chain(x, img, nxt.features[0] if isinstance(nxt, QuantizedBlock) else None)
            else:
                x, img = m(x), None
        return self.fc(self.flattener(self.avgpool(x)))


def resnet18_approx(weights=None, bn_stats_batches=0, device=None, **cfg):
    fp = ResNet(BasicBlock, (2, 2, 2, 2))
    if weights:
        load_float_weights(fp, weights)
    elif bn_stats_batches:
        estimate_bn_statistics(fp, bn_stats_batches, device=device)
    return QuantizedResNet(fp, **approx_qparams(**cfg))


def resnet50_approx(weights=None, bn_stats_batches=0, device=None, **cfg):
    fp = ResNet(Bottleneck, (3, 4, 6, 3))
    if weights:
        load_float_weights(fp, weights)
    elif bn_stats_batches:
        estimate_bn_statistics(fp, bn_stats_batches, device=device)
    return QuantizedResNet(fp, **approx_qparams(**cfg))


def approx_layer_shapes(model, image_hw=224):
    """(name, M_per_image, K, N, groups) of every approx product for one image."""
    shapes, hooks = [], []

    def conv_hook(mod, inp, out):
        cog = mod.out_channels // mod.groups
        K = (mod.in_channels // mod.groups) * mod.kernel_size[0] * mod.kernel_size[1]
        shapes.append((type(mod).__name__, out.shape[2] * out.shape[3], K, cog, mod.groups))

    def lin_hook(mod, inp, out):  # rows per image: 1 for [B, K], T for token inputs [B, T, K]
        rows = inp[0].numel() // (mod.in_features * inp[0].shape[0])
        shapes.append((type(mod).__name__, rows, mod.in_features, mod.out_features, 1))

    for m in model.modules():
        if isinstance(m, QCustomBNConv2dTorch):
            hooks.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, QCustomLinearTorch):
            hooks.append(m.register_forward_hook(lin_hook))
    return shapes, hooks


def approx_macs_per_image(shapes):
    return sum(Mi * K * N * g for (_, Mi, K, N, g) in shapes)
