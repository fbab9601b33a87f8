"""Host logic that runs without a GPU: error-table selection (v9:555-592), flag words,
operator configuration plumbing and the reference's exception conventions."""
import numpy as np
import pytest
import torch
from torch import nn

from fp8_quantization_amd import _lib
from fp8_quantization_amd.approx_ops import make_flags
from fp8_quantization_amd.error_tables import get_error_table_NN
from tests import golden_io as gio


@pytest.mark.parametrize("E,M,wc,dn,key", [
    (4, 3, True, 3, "E4M3_table_comp"), (4, 3, False, 3, "E4M3_table_nocomp"), (4, 3, False, 7, "E4M3_table_nocomp"),
    (3, 4, True, 3, "E3M4_table_comp3"), (3, 4, True, 4, "E3M4_table_comp4"), (3, 4, True, 9, "E3M4_table_comp4"),
    (3, 4, False, 3, "E3M4_table_nocomp"), (2, 5, True, 3, "E2M5_table_comp3"), (2, 5, True, 4, "E2M5_table_comp4"),
    (2, 5, True, 5, "E2M5_table_comp5"), (2, 5, False, 5, "E2M5_table_nocomp")])
def test_error_table_selection_matches_reference(E, M, wc, dn, key):
    g = gio.load("g2_matmul.npz")
    np.testing.assert_array_equal(get_error_table_NN(E, M, wc, dn).numpy(), g[key])


def test_error_table_quirks():
    with pytest.raises(ValueError):
        get_error_table_NN(5, 2, True, 3)          # E5M2 unsupported by the reference (F3)
    with pytest.raises(UnboundLocalError):
        get_error_table_NN(3, 4, True, 2)          # unlisted dnsmp_factor (F3)
    with pytest.raises(UnboundLocalError):
        get_error_table_NN(2, 5, True, 6)


def test_flag_words_match_header():
    assert make_flags(True, True, True, True, True) == 31
    assert make_flags(False, False, False, False) == 0
    assert make_flags(with_approx=True, with_s2nn2s_opt=False, quant_btw_mult_accu=True) == _lib.APPROX | _lib.QBMA


def _qparams(approx=True, res=True, E=4, M=3):
    from fp8_quantization_amd.quantization import FPQuantizer, RangeEstimators
    return dict(method=FPQuantizer, act_method=FPQuantizer, n_bits=8, per_channel_weights=True,
                weight_range_method=RangeEstimators.current_minmax.cls,
                act_range_method=RangeEstimators.allminmax.cls, quantize_input=True,
                fp8_kwargs=dict(maxval=None, mantissa_bits=M, set_maxval=True),
                custom_approx_params=dict(expo_width=E, mant_width=M, dnsmp_factor=3, withComp=False,
                                          with_approx=True, with_s2nn2s_opt=True, sim_hw_add_OFUF=False,
                                          with_OF_opt=False, with_UF_opt=False, golden_clip_OF=False,
                                          quant_btw_mult_accu=True, debug_mode=False, self_check_mode=False),
                run_method=dict(approx_flag=approx, quantize_after_mult_and_add=False, res_quantizer_flag=res,
                                original_quantize_res=False))


def test_operator_construction_contract():
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
    conv = QCustomBNConv2dTorch(in_channels=4, out_channels=8, kernel_size=3, padding=1, bias=False,
                                activation=nn.ReLU(), **_qparams())
    assert conv.bias is None and conv.gamma.shape == (8,) and conv.approx_flag
    lin = QCustomLinearTorch(in_features=16, out_features=10, bias=True, **_qparams())
    assert lin.weight.shape == (10, 16)
    assert conv.custom_approx_params["mant_width"] == 3


def test_approx_without_res_quantizer_raises_value_error():
    from fp8_quantization_amd.approx_calculation import QCustomLinearTorch
    lin = QCustomLinearTorch(in_features=4, out_features=3, bias=False, **_qparams(approx=True, res=False))
    lin.run_forward = lambda x, w, b, offsets=None: x @ w.t()  # host-only stand-in: no device work
    with pytest.raises(ValueError):
        lin(torch.randn(2, 4))


def test_unsupported_format_raises_before_device_work():
    from fp8_quantization_amd.approx_calculation import QCustomLinearTorch
    lin = QCustomLinearTorch(in_features=4, out_features=3, bias=False, **_qparams(E=5, M=2))
    with pytest.raises(ValueError):
        lin.approx_multiply(torch.randn(2, 4), torch.randn(4, 3), None, torch.zeros(3), None)


def test_three_d_linear_input_asserts_like_reference():
    from fp8_quantization_amd.approx_calculation import QCustomLinearTorch
    lin = QCustomLinearTorch(in_features=4, out_features=3, bias=False, **_qparams())
    with pytest.raises(AssertionError):
        lin.run_forward(torch.randn(2, 5, 4), lin.weight, None)


def test_cpu_tensors_are_rejected_not_computed():
    from fp8_quantization_amd import approx_matmul
    with pytest.raises(RuntimeError):
        approx_matmul(torch.ones(2, 3), torch.ones(3, 2), 4, 3, 7, 7, 7, None, with_approx=True)


def test_quantized_mobilenet_v2_matches_reference_module_tree():
    """The module swap (fold_bn / quantize_sequential / quantize_model) applied to the float
    MobileNetV2 gives the reference QuantizedMobileNetV2's exact state_dict layout (G8)."""
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    c = gio.meta()["g8"][0]
    g = gio.load("g8_mbv2.npz")
    m = mobilenet_v2_approx(input_size=c["input_size"], width_mult=c["width_mult"], n_class=c["n_class"],
                            expo_width=c["E"], mant_width=c["M"], withComp=c["with_comp"])
    sd = m.state_dict()
    assert set(sd) == set(c["state_keys"])
    for k in c["state_keys"]:
        assert tuple(sd[k].shape) == g[f"{c['name']}__state__{k}"].shape, k
    names = [n for n, mod in m.named_modules() if isinstance(mod, (QCustomBNConv2dTorch, QCustomLinearTorch))]
    assert names == c["approx_layers"]


def test_module_swap_rejects_layers_outside_the_approx_path():
    import pytest
    from torch import nn

    from fp8_quantization_amd.model_wrap import quantize_model
    from fp8_quantization_amd.resnet_workload import approx_qparams
    with pytest.raises(NotImplementedError):
        quantize_model(nn.Sequential(nn.Conv1d(3, 4, 3)), **approx_qparams())


def test_bn_act_epilogue_eligibility_and_parameters():
    """BNFusedHijacker hands BN + clamp activation to the kernel only in the single-product
    eval form (quantized_folded_bn.py module doc); the scale/shift pair is ATen's eval transform."""
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch
    from fp8_quantization_amd.approx_ops import bn_act_epilogue
    conv = QCustomBNConv2dTorch(in_channels=4, out_channels=8, kernel_size=3, padding=1, bias=False,
                                activation=nn.ReLU6(), **_qparams())
    with torch.no_grad():
        conv.running_mean.uniform_(-1, 1)
        conv.running_var.uniform_(0.5, 2)
        conv.gamma.uniform_(0.5, 1.5)
        conv.beta.uniform_(-1, 1)
    conv.eval()
    assert conv._fused_epilogue() is None            # ranges not fixed yet
    conv.fix_ranges_flag = True
    ss, act, lo, hi = conv._fused_epilogue()
    assert (act, lo, hi) == (1, 0.0, 6.0) and ss.shape == (8, 2)
    y = torch.randn(3, 8, 5, 5)
    bn = torch.nn.functional.batch_norm(y, conv.running_mean, conv.running_var, conv.gamma, conv.beta, False, 0.1,
                                        conv.epsilon)
    torch.testing.assert_close(y * ss[:, 0].view(1, -1, 1, 1) + ss[:, 1].view(1, -1, 1, 1), bn, rtol=1e-5,
                               atol=1e-5)
    conv.train()
    assert conv._fused_epilogue() is None
    conv.eval()
    conv.original_quantize_res = True
    assert conv._fused_epilogue() is None
    conv.original_quantize_res = False
    conv.fuse_bn_act = False
    assert conv._fused_epilogue() is None
    conv.fuse_bn_act = True
    conv.activation_function = nn.GELU()
    assert conv._fused_epilogue() is None            # not a clamp: BN + GELU stay unfused
    assert bn_act_epilogue(conv.running_mean, conv.running_var, None, None, 1e-5, nn.ReLU())[1:] == \
        (1, 0.0, float("inf"))


def test_fix_ranges_error_semantics_match_reference():
    """quantization_manager.py:93-98: fixing the ranges of a quantizer that is not initialized
    raises QuantizerNotInitializedError (quantizers/utils.py:6-12); the model-wide fix
    (base_quantized_classes.py:23-28) skips such managers.  The FP8 quantizer reports itself
    initialized from construction on (fp8_quantizer.py:252-254), so its managers always fix."""
    from fp8_quantization_amd.quantization import FPQuantizer, QuantizationManager, QuantizerNotInitializedError, Qstates
    from fp8_quantization_amd.quantization.base_quantized_classes import _set_layer_fix_ranges

    class Uninit(FPQuantizer):
        @property
        def is_initialized(self):
            return False

    mgr = QuantizationManager(qmethod=Uninit, qparams=dict(mantissa_bits=3))
    with pytest.raises(QuantizerNotInitializedError, match="not been initialized"):
        mgr.fix_ranges()
    assert mgr.state == Qstates.estimate_ranges
    _set_layer_fix_ranges(mgr)  # skipped, no raise
    assert mgr.state == Qstates.estimate_ranges
    ok = QuantizationManager(qmethod=FPQuantizer, qparams=dict(mantissa_bits=3))
    assert ok.quantizer.is_initialized
    ok.fix_ranges()
    assert ok.state == Qstates.fix_ranges and ok.quantizer.state == Qstates.fix_ranges
