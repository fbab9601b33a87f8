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


def _oracle_sum_abs(mod, x, w, E, M, tab, flags, bA, bB, bR, approx):
    """Sum_k |v_k| per output of the layer's product on the reference's operands: the oracle's
    terms (per group, im2col, single-output-channel groups with the tensor-bias semantics) for an
    approx product, |a * b| for the exact one; [rows, N] in the output's NCHW-flattened order."""
    import torch.nn.functional as F
    from oracle import oracle as orc
    tab = np.ascontiguousarray(tab, np.int32)
    if w.dim() == 2:  # linear: x [B, K] @ w^T
        A, B = x, w.t().contiguous()
        if not approx:
            return np.abs(A.numpy()).astype(np.float64) @ np.abs(B.numpy()).astype(np.float64)
        return orc.matmul(A.numpy(), B.numpy(), E, M, int(bA[0]), bB, int(bR[0]), tab, flags, with_abs=True)[1]
    g = mod.groups
    cin_g, cout_g = x.shape[1] // g, w.shape[0] // g
    sums = []
    for j in range(g):
        cols = F.unfold(x[:, j * cin_g:(j + 1) * cin_g], w.shape[2:], dilation=mod.dilation, padding=mod.padding,
                        stride=mod.stride)
        A = cols.transpose(1, 2).reshape(-1, cols.shape[1]).numpy()
        B = w[j * cout_g:(j + 1) * cout_g].reshape(cout_g, -1).t().contiguous().numpy()
        if not approx:
            sums.append(np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64))
            continue
        tb = orc.TB if cout_g == 1 else 0  # approx_calculation.py:800-809
        sums.append(orc.matmul(A, B, E, M, int(bA[0]), bB[j * cout_g:(j + 1) * cout_g], int(bR[0]), tab, flags | tb,
                               with_abs=True)[1])
    return np.concatenate(sums, axis=1)


@pytest.mark.parametrize("case", gio.meta()["g8"], ids=lambda c: c["name"])
def test_mobilenet_v2_layers_teacher_forced(case):
    """Every approx layer of the reference's own QuantizedMobileNetV2 forward, teacher-forced:
    the engine's run_forward (the drop-in surface, approx_calculation.py:822-917 / 1007-1023) on
    exactly the quantized input and weight the reference's run_forward received (G8's per-layer
    records) must return the reference's product within north_star's 1e-5 * sum_k |v_k| (sum
    from the oracle's terms on the same operands; |a b| for the exact product of config 1); and the
    layer's whole forward on the reference's recorded layer input (the fused input quantizer, BN
    and activation in the store) must land within the BN-scaled bar of the reference's layer
    output."""
    from fp8_quantization_amd.approx_calculation import QCustomBNConv2dTorch
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    g = gio.load("g8_mbv2.npz")
    name = case["name"]
    approx = case["run_method"]["approx_flag"]
    m = mobilenet_v2_approx(input_size=case["input_size"], width_mult=case["width_mult"], n_class=case["n_class"],
                            expo_width=case["E"], mant_width=case["M"], withComp=case["with_comp"],
                            run_method=case.get("run_method"), zero_table_ext=case.get("zero_table_ext", False))
    state = {k: torch.from_numpy(g[f"{name}__state__{k}"]) for k in case["state_keys"]}
    torch.nn.Module.load_state_dict(m, state, strict=True)
    m = m.to(DEV).eval()
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.from_numpy(g[f"{name}__x_cal"]).to(DEV))
    m.fix_ranges()
    mods = dict(m.named_modules())
    worst = 0.0
    for lname in case["approx_layers"]:
        mod = mods[lname]
        L = lambda k: torch.from_numpy(g[f"{name}__L__{lname}__{k}"])  # noqa: E731
        x, w, y_ref = L("x"), L("w"), L("y").numpy().astype(np.float64)
        bA, bB, bR = (g[f"{name}__{k}__{lname}"] for k in ("bA", "bB", "bR"))
        for key, get, want in (("bA", mod.get_acts_fp_bias, bA), ("bB", mod.get_weights_fp_bias, bB),
                               ("bR", mod.get_res_fp_bias, bR)):
            np.testing.assert_array_equal(get().reshape(-1).cpu().numpy(), want, err_msg=f"{lname} {key}")
        E, M, tab, flags = mod._approx_config()
        bias = None if getattr(mod, "bias", None) is None else mod.bias.detach()
        with torch.no_grad():
            y = mod.run_forward(x.to(DEV), w.to(DEV), bias).cpu().numpy().astype(np.float64)
        assert y.shape == y_ref.shape, lname
        S = _oracle_sum_abs(mod, x, w, E, M, tab.numpy(), int(flags), bA.astype(np.int32), bB.astype(np.int32),
                            bR.astype(np.int32), approx)
        if y.ndim == 4:  # NCHW -> [rows, channels], the oracle's layout
            y, y_ref = (t.transpose(0, 2, 3, 1).reshape(-1, t.shape[1]) for t in (y, y_ref))
        tol = gio.sum_tolerance(S.astype(np.float64))
        bad = np.abs(y - y_ref) > tol
        assert not bad.any(), f"{lname}: {np.count_nonzero(bad)} of {y.size} product outputs outside 1e-5 sum|v|"
        worst = max(worst, float(np.max(np.abs(y - y_ref) / np.maximum(tol, 1e-30))))
        if approx and isinstance(mod, QCustomBNConv2dTorch):  # the layer's own fused forward
            with torch.no_grad():
                out = mod(L("in").to(DEV)).cpu().numpy().astype(np.float64)
            out_ref = L("out").numpy().astype(np.float64)
            sc = (mod.gamma / torch.sqrt(mod.running_var + mod.epsilon)).detach().cpu().numpy().astype(np.float64)
            out, out_ref = (t.transpose(0, 2, 3, 1).reshape(-1, t.shape[1]) for t in (out, out_ref))
            mean_sc = np.abs(mod.running_mean.detach().cpu().numpy().astype(np.float64) * sc)
            beta = np.abs(mod.beta.detach().cpu().numpy().astype(np.float64))
            # (F.batch_norm's (x - mean) * invstd * gamma + beta vs the store's fma(acc, scale, shift):
            # a few fp32 roundings of the intermediates apart)
            bar = np.abs(sc)[None, :] * tol + 8 * 2.0 ** -24 * (np.abs(out_ref) + np.abs(y_ref * sc[None, :])
                                                                 + (mean_sc + beta)[None, :] + 1e-30)
            bad = np.abs(out - out_ref) > bar
            assert not bad.any(), f"{lname}: {np.count_nonzero(bad)} layer outputs outside the BN-scaled bar"
    print(f"{name}: worst |y - y_ref| / bar = {worst:.3g} over {len(case['approx_layers'])} layers")
