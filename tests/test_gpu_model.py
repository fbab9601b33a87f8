"""Model-level parity (G8): the reference's QuantizedMobileNetV2 (width 0.25, 32x32, random
weights and BN statistics) rebuilt from the drop-in operators, given the reference's initial
state, goes through estimate -> fix -> approx on the GPU.  Cases: E4M3 approx_v9; E4M3 with
approx_flag off (BASELINE config 1: the reference's canonical --no-approx_flag
--original-quantize-res run, exact product + quantizers); E5M2 approx_v9 with the opt-in zero
table (BASELINE config 3's format; the reference was given the same zero table).  In the
no-approx case the exact products (groups = 1) run on the bf16 matrix core (dn_gemm_bf16)
(csrc/gemm_dense.h), the depthwise ones on fp8a_grouped_conv2d: no torch / MIOpen convolution
runs in that forward.

Bars: every approx layer's bA / per-channel bB / bR identical (calibration reproduced through
the whole network); logits within a summation-order tolerance; top-1 identical."""
import numpy as np
import pytest
import torch

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("case", gio.meta()["g8"], ids=lambda c: c["name"])
def test_mobilenet_v2_model_level(case, monkeypatch):
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    g = gio.load("g8_mbv2.npz")
    name = case["name"]
    m = mobilenet_v2_approx(input_size=case["input_size"], width_mult=case["width_mult"], n_class=case["n_class"],
                            expo_width=case["E"], mant_width=case["M"], withComp=case["with_comp"],
                            run_method=case.get("run_method"), zero_table_ext=case.get("zero_table_ext", False))
    state = {k: torch.from_numpy(g[f"{name}__state__{k}"]) for k in case["state_keys"]}
    missing, unexpected = torch.nn.Module.load_state_dict(m, state, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    m = m.to(DEV).eval()
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.from_numpy(g[f"{name}__x_cal"]).to(DEV))
    m.fix_ranges()
    from fp8_quantization_amd import _lib
    _lib.path_stats(reset=True)
    if not case["run_method"]["approx_flag"]:  # config 1: every product on the HIP kernels
        def no_torch_conv(*a, **k):
            raise AssertionError("torch convolution in the config-1 forward")
        monkeypatch.setattr(torch.nn.functional, "conv2d", no_torch_conv)
    with torch.no_grad():
        logits = m(torch.from_numpy(g[f"{name}__x_ev"]).to(DEV)).cpu().numpy()
    monkeypatch.undo()
    paths = _lib.path_stats(reset=True)
    if not case["run_method"]["approx_flag"]:  # config 1: the exact products on the fp8 matrix core
        assert paths["dense"] > 0 and paths["f8mx"] == 0, paths
    mods = dict(m.named_modules())
    for lname in case["approx_layers"]:
        mod = mods[lname]
        assert isinstance(mod, (QCustomBNConv2dTorch, QCustomLinearTorch))
        for key, get in (("bA", mod.get_acts_fp_bias), ("bB", mod.get_weights_fp_bias), ("bR", mod.get_res_fp_bias)):
            np.testing.assert_array_equal(get().reshape(-1).cpu().numpy(), g[f"{name}__{key}__{lname}"],
                                          err_msg=f"{lname} {key}")
    ref = g[f"{name}__logits"]
    assert logits.shape == ref.shape
    assert np.max(np.abs(logits - ref)) <= 1e-3 * np.abs(ref).max(), np.max(np.abs(logits - ref))
    assert np.array_equal(logits.argmax(1), ref.argmax(1))
