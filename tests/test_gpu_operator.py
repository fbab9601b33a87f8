"""Operator-level parity (G5): the drop-in QCustomBNConv2dTorch / QCustomLinearTorch, built with
the reference's constructor contract and fed the same state, go through estimate -> fix ->
approx exactly like the reference modules did when tests/golden/g5_operator.npz was recorded.

Biases (bA, per-channel bB, bR) must match exactly; outputs (post BN + ReLU for convs) within
a summation-order tolerance scaled by the output magnitude.
"""
import numpy as np
import pytest
import torch
from torch import nn

from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
META = gio.meta()


def _build(case, qp):
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch, QCustomLinearTorch
    shp = case["shape"]
    if "fin" in shp:
        return QCustomLinearTorch(in_features=shp["fin"], out_features=shp["fout"], bias=True, **qp)
    return QCustomBNConv2dTorch(in_channels=shp["cin"], out_channels=shp["cout"], kernel_size=shp["k"],
                                stride=shp["stride"], padding=shp["pad"], groups=shp["groups"], bias=False,
                                activation=nn.ReLU(), **qp)


@pytest.mark.parametrize("case", META["g5"], ids=lambda c: c["name"])
def test_operator_estimate_fix_approx(case):
    from fp8_quantization_amd.resnet_workload import approx_qparams
    g = gio.load("g5_operator.npz")
    name = case["name"]
    qp = approx_qparams(expo_width=case["E"], mant_width=case["M"], dnsmp_factor=3, withComp=case["with_comp"],
                        with_s2nn2s_opt=case["s2n"], quant_btw_mult_accu=case["qbma"],
                        run_method=case.get("run_method"))
    mod = _build(case, qp)
    state = {k: torch.from_numpy(g[f"{name}__state__{k}"]) for k in case["state_keys"]}
    missing, unexpected = mod.load_state_dict(state, strict=False)
    assert not unexpected, unexpected
    mod = mod.to(DEV).eval()
    mod.quantized()
    mod.estimate_ranges()
    with torch.no_grad():
        y_cal = mod(torch.from_numpy(g[f"{name}__x_cal"]).to(DEV))
    mod.fix_ranges()
    with torch.no_grad():
        y_ev = mod(torch.from_numpy(g[f"{name}__x_ev"]).to(DEV))
    np.testing.assert_array_equal(mod.get_acts_fp_bias().reshape(-1).cpu().numpy(), g[f"{name}__bA"])
    np.testing.assert_array_equal(mod.get_weights_fp_bias().reshape(-1).cpu().numpy(), g[f"{name}__bB"])
    np.testing.assert_array_equal(mod.get_res_fp_bias().reshape(-1).cpu().numpy(), g[f"{name}__bR"])
    for got, key in ((y_cal, "y_cal"), (y_ev, "y_ev")):
        ref = g[f"{name}__{key}"]
        got = got.cpu().numpy()
        assert got.shape == ref.shape
        scale = np.abs(ref).max() + 1e-30
        assert np.max(np.abs(got - ref)) <= 1e-5 * scale * max(1, ref.shape[1]), (key, np.max(np.abs(got - ref)))
