"""fp8a_grouped_conv2d -- the exact grouped / depthwise convolution (QCustomConv2dTorch's per-group
im2col + x @ w^T, approx_calculation.py:686-711; the exact branch's x @ y[:, i] for groups > 1,
:797; BASELINE config 1's depthwise layers) against the same im2col product in float64.

Bar: |y - ref| <= 1e-5 * sum |x w| per output (fp32 FMAs in im2col k order vs an exact sum); the
padding is read as zeros, so a non-finite weight gives NaN exactly where the im2col product does."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def im2col_ref(x, w, groups, stride, padding, dilation):
    """The reference's per-group im2col product in float64 (approx_calculation.py:686-711)."""
    Bn, Cin, H, W = x.shape
    Cout, cig, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    col = F.unfold(x.double(), (kh, kw), dilation=dilation, padding=padding, stride=stride)  # [Bn, Cin kh kw, L]
    col = col.transpose(1, 2).reshape(Bn * Ho * Wo, Cin * kh * kw)
    wc = w.double().reshape(Cout, -1)
    cog, kg = Cout // groups, cig * kh * kw
    out, mag = [], []
    for g in range(groups):
        a = col[:, g * kg:(g + 1) * kg]
        b = wc[g * cog:(g + 1) * cog].T
        out.append(a @ b)
        mag.append(a.abs() @ b.abs())
    to_nchw = lambda t: torch.cat(t, 1).reshape(Bn, Ho, Wo, Cout).permute(0, 3, 1, 2)  # noqa: E731
    return to_nchw(out), to_nchw(mag)


CASES = [  # (Bn, Cin, H, W, Cout, groups, k, stride, padding, dilation)
    (2, 32, 14, 14, 32, 32, 3, 1, 1, 1),    # MobileNetV2 depthwise, stride 1
    (2, 24, 15, 13, 24, 24, 3, 2, 1, 1),    # stride 2, odd sizes (Wo not a multiple of 4)
    (1, 16, 9, 11, 16, 16, 5, 2, 2, 1),     # 5x5
    (1, 16, 10, 10, 32, 16, 3, 1, 1, 1),    # depth multiplier 2
    (2, 6, 12, 12, 8, 2, 3, 1, 2, 2),       # groups of 3 input channels, dilation 2 (general loop)
    (1, 8, 7, 7, 8, 4, 1, 1, 0, 1),         # 1x1 grouped
    (1, 4, 20, 20, 4, 4, 7, 3, 3, 1),       # 7x7 stride 3 (general loop)
    (3, 1, 5, 6, 2, 1, 3, 1, 1, 1),         # groups 1
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_grouped_conv_matches_im2col(case):
    from fp8_quantization_amd.approx_ops import grouped_conv2d
    Bn, Cin, H, W, Cout, groups, k, s, p, d = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(Bn, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin // groups, k, k, generator=g)
    y = grouped_conv2d(x.to(DEV), w.to(DEV), groups, (s, s), (p, p), (d, d)).cpu().double()
    ref, mag = im2col_ref(x, w, groups, (s, s), (p, p), (d, d))
    assert y.shape == ref.shape
    assert torch.all((y - ref).abs() <= 1e-5 * mag + 1e-30)


def test_grouped_conv_fp8_values_exact_order():
    """FP8 (E4M3) operands on a depthwise 3x3: fp32 FMAs in k order equal the fp32 im2col sum in
    the same order to the bit (each product is exact in fp32)."""
    from fp8_quantization_amd.approx_ops import grouped_conv2d
    g = torch.Generator().manual_seed(7)
    q = lambda t: t.to(torch.float8_e4m3fn).float()  # noqa: E731
    x, w = q(torch.randn(2, 8, 9, 9, generator=g) * 4), q(torch.randn(8, 1, 3, 3, generator=g))
    y = grouped_conv2d(x.to(DEV), w.to(DEV), 8, (1, 1), (1, 1), (1, 1)).cpu()
    col = F.unfold(x, (3, 3), padding=1).reshape(2, 8, 9, 81)  # [Bn, C, k, L]
    acc = torch.zeros(2, 8, 81)
    for kk in range(9):  # fp32, k order
        acc = acc + col[:, :, kk, :] * w.reshape(8, 9)[None, :, kk, None]
    assert torch.equal(y.reshape(2, 8, 81), acc)


def test_grouped_conv_nonfinite_weight_like_im2col():
    from fp8_quantization_amd.approx_ops import grouped_conv2d
    x = torch.rand(1, 4, 6, 6) + 0.5
    w = torch.rand(4, 1, 3, 3)
    w[1, 0, 0, 0] = float("inf")
    y = grouped_conv2d(x.to(DEV), w.to(DEV), 4, (1, 1), (1, 1), (1, 1)).cpu()
    ref, _ = im2col_ref(x, w, 4, (1, 1), (1, 1), (1, 1))
    assert torch.equal(torch.isnan(y), torch.isnan(ref))  # 0 (padding) * inf in the top row / left column
    assert torch.isnan(y[0, 1, 0, :]).all() and torch.isinf(y[0, 1, 1:, 1:]).all()


def test_grouped_conv_empty_batch_and_errors():
    from fp8_quantization_amd.approx_ops import grouped_conv2d
    y = grouped_conv2d(torch.zeros(0, 4, 5, 5, device=DEV), torch.ones(4, 1, 3, 3, device=DEV), 4, (1, 1), (1, 1))
    assert y.shape == (0, 4, 5, 5)
    with pytest.raises(AssertionError):
        grouped_conv2d(torch.zeros(1, 6, 5, 5, device=DEV), torch.ones(4, 1, 3, 3, device=DEV), 4)


def test_exact_conv_module_routes_to_hip():
    """QCustomConv2dTorch with groups > 1 runs fp8a_grouped_conv2d (a dense-path launch), never
    torch's convolution (the no-approx QCustomBNConv2dTorch depthwise layers: test_gpu_model.py)."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_calculation import QCustomConv2dTorch
    m = QCustomConv2dTorch(8, 8, 3, padding=1, groups=8, bias=True).to(DEV).eval()
    x = torch.randn(2, 8, 10, 10, device=DEV)
    _lib.path_stats(reset=True)
    orig = F.conv2d
    try:
        F.conv2d = lambda *a, **k: (_ for _ in ()).throw(AssertionError("torch convolution"))
        y = m.run_forward(x, m.weight, m.bias)
    finally:
        F.conv2d = orig
    assert _lib.path_stats(reset=True)["dense"] == 1
    ref = orig(x.cpu().double(), m.weight.detach().cpu().double(), m.bias.detach().cpu().double(), 1, 1, 1, 8)
    assert torch.allclose(y.cpu().double(), ref, atol=1e-5, rtol=1e-5)


def _fma_bn(r, scale, shift):
    return (r.double() * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1)).float()


@pytest.mark.parametrize("groups,cin,cout,k,s", [(16, 16, 16, 3, 1), (24, 24, 24, 3, 2), (1, 8, 24, 1, 1), (1, 6, 10, 3, 2)])
@pytest.mark.parametrize("order", ["in_res", "out"])
def test_config1_fused_layer(groups, cin, cout, k, s, order):
    """fp8a_dense_conv2d_fused (BASELINE config 1's layer in one pass) against its stages run
    separately on the same kernels: fq_in (quantize_input) -> exact conv -> fq_res -> scale / shift
    -> clamp, or conv -> scale / shift -> clamp -> fq_out; the biases are the quantizers' own."""
    from fp8_quantization_amd.approx_ops import (dense_conv2d, dense_conv2d_fused, dense_format, fp8_fake_quantize,
                                                 grouped_conv2d)
    g = torch.Generator().manual_seed(groups + cin + cout + k + s)
    x = (torch.randn(2, cin, 13, 13, generator=g) * 2).relu().to(DEV)
    w = (torch.randn(cout, cin // groups, k, k, generator=g) * 0.3).to(DEV)
    w, _ = fp8_fake_quantize(w, torch.tensor([2.0]), 8, 3)
    scale = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    ep = torch.stack((scale, shift), 1).contiguous()
    mxi, mxr, mxo = torch.tensor([6.0], device=DEV), torch.tensor([40.0], device=DEV), torch.tensor([6.0], device=DEV)
    pad = k // 2
    conv = (lambda t: grouped_conv2d(t, w, groups, (s, s), (pad, pad))) if groups > 1 else \
        (lambda t: dense_conv2d(t, w, dense_format(3), (s, s), (pad, pad)))
    if order == "in_res":
        y, b = dense_conv2d_fused(x, w, groups, (s, s), (pad, pad), qin=(mxi, 8, 3, 1), rq=(mxr, 8, 3, 1),
                                  bn=(ep, 1, 0.0, 6.0))
        xq, bi = fp8_fake_quantize(x, mxi, 8, 3)
        r, br = fp8_fake_quantize(conv(xq), mxr, 8, 3)
        ref = torch.clamp(_fma_bn(r, scale, shift), 0.0, 6.0)
        assert torch.equal(b["qin"], bi) and torch.equal(b["rq"], br)
    else:
        y, b = dense_conv2d_fused(x, w, groups, (s, s), (pad, pad), bn=(ep, 1, 0.0, 6.0), oq=(mxo, 8, 3, 1))
        r = conv(x)
        ref, bo = fp8_fake_quantize(torch.clamp(_fma_bn(r, scale, shift), 0.0, 6.0), mxo, 8, 3)
        assert torch.equal(b["oq"], bo)
    # the scale / shift is one fma on both sides (float64 then float32 stands in for it); the sums
    # of the two paths are the same kernels' -- equal but for rare double-rounding last bits
    d = (y - ref).abs()
    assert (d == 0).float().mean() > 0.999
    assert torch.all(d <= 1e-6 * ref.abs() + 1e-12)


@pytest.mark.parametrize("groups,cin,cout,k,s,bn_", [(1, 8, 24, 1, 1, 2), (1, 6, 10, 3, 2, 2), (16, 16, 16, 3, 1, 2),
                                                  (24, 24, 24, 3, 2, 2), (4, 8, 12, 3, 1, 2), (1, 8, 24, 1, 1, 0),
                                                  (16, 16, 16, 3, 1, 0)])
@pytest.mark.parametrize("per_channel", [False, True])
def test_config1_fused_weight_quantizer(groups, cin, cout, k, s, bn_, per_channel):
    """The weight quantizer inside the fused layer (fp8a_dense_conv2d_fused's w_maxval: applied to
    every weight as the product loads it) against the weights quantized first by fp8a_fp8_quantize:
    the same bits out, and the same custom_bias ([1], or [Cout, 1, 1, 1] per channel) -- on the
    dense product, the LDS depthwise kernel, the general grouped kernel, and an empty batch (no
    product: the biases still written)."""
    from fp8_quantization_amd.approx_ops import dense_conv2d_fused, fp8_fake_quantize
    g = torch.Generator().manual_seed(groups + cin + cout + k + s + per_channel)
    x = (torch.randn(bn_, cin, 11, 12, generator=g) * 2).relu().to(DEV)
    w = (torch.randn(cout, cin // groups, k, k, generator=g) * 0.3).to(DEV)
    mxw = (torch.rand(cout, generator=g) + 0.2 if per_channel else torch.tensor([0.7])).to(DEV)
    wq, bw = fp8_fake_quantize(w, mxw, 8, 3, per_row=per_channel)
    scale = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    ep = torch.stack((scale, shift), 1).contiguous()
    kw = dict(qin=(torch.tensor([6.0], device=DEV), 8, 3, 1), rq=(torch.tensor([40.0], device=DEV), 8, 3, 1),
              bn=(ep, 1, 0.0, 6.0))
    pad = k // 2
    y_ref, b_ref = dense_conv2d_fused(x, wq, groups, (s, s), (pad, pad), **kw)
    y, b = dense_conv2d_fused(x, w, groups, (s, s), (pad, pad), wq=(mxw, 8, 3, 1), **kw)
    assert torch.equal(y, y_ref)
    assert b["wq"].shape == bw.shape and torch.equal(b["wq"], bw)
    assert torch.equal(b["wq"]._fp8a_i32.cpu(), bw._fp8a_i32.cpu())
    assert torch.equal(b["qin"], b_ref["qin"]) and torch.equal(b["rq"], b_ref["rq"])


def test_dense_marks_tagged_per_call():
    """The dense path's fallback marks carry a per-call tag instead of being cleared: a call that
    marks every unit (fp32 operands off the bf16 grid, all recomputed by dn_fix) followed, in the
    same workspace, by calls that mark none and some -- each against the float64 product."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_conv2d, dense_format
    g = torch.Generator().manual_seed(5)
    w = (torch.randn(70, 9, 3, 3, generator=g) * 0.3).bfloat16().float()
    xs = [torch.randn(2, 9, 20, 20, generator=g), torch.randn(2, 9, 20, 20, generator=g).bfloat16().float()]
    x3 = xs[1].clone()
    x3[1, 4, 7, 7] = 1.0 + 2.0 ** -20  # one unit off the grid
    xs.append(x3)
    _lib.dense_stats(reset=True)
    for x in xs:
        y = dense_conv2d(x.to(DEV), w.to(DEV), dense_format(3), (1, 1), (1, 1))
        ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1)
        assert torch.allclose(y.cpu().double(), ref, atol=1e-4, rtol=1e-5)
    assert _lib.dense_stats()["fp32_launches"] == 2  # the first and third calls recomputed units; the second none


DW3_SHAPES = [  # (Bn, C, H, W, stride, padding): every MobileNetV2 depthwise geometry + ragged ones
    (2, 32, 112, 112, 1, 1), (2, 96, 112, 112, 2, 1), (2, 144, 56, 56, 1, 1), (2, 144, 56, 56, 2, 1),
    (3, 192, 28, 28, 1, 1), (3, 192, 28, 28, 2, 1), (4, 384, 14, 14, 1, 1), (4, 576, 14, 14, 2, 1),
    (5, 960, 7, 7, 1, 1), (1, 3, 5, 9, 1, 1), (2, 5, 13, 7, 2, 1), (1, 4, 9, 300, 1, 1), (1, 6, 11, 10, 1, 0),
    (2, 7, 12, 13, 2, 2), (1, 2, 1, 1, 1, 1),
]


@pytest.mark.parametrize("shape", DW3_SHAPES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("form", [1, 2])
def test_depthwise_lds_form_matches_general_kernel(shape, fused, form):
    """The LDS-staged depthwise 3x3 (option "dw3" = 1: register-staged dn_dw3_kernel; 2: the
    LDS-DMA-staged dn_dw3g_kernel) against the general dn_group_conv (dw3 = 0): the same fp32 FMAs
    in the same order, so the same bits -- bands of
    rows and groups of whole planes, ragged rows, stride 2, padding 0 / 2, a single-pixel plane,
    non-finite weights, and the config-1 tail (qin on load, rq, scale / shift, clamp)."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_conv2d_fused, fp8_fake_quantize, grouped_conv2d
    Bn, C, H, W, s, p = shape
    g = torch.Generator().manual_seed(Bn * C + H * W + s)
    x = (torch.randn(Bn, C, H, W, generator=g) * 2).to(DEV)
    w = torch.randn(C, 1, 3, 3, generator=g)
    w[0, 0, 1, 1] = float("inf")
    w[-1, 0, 2, 0] = float("nan")
    w = w.to(DEV)

    def run():
        if not fused:
            return grouped_conv2d(x, w, C, (s, s), (p, p))
        wq, _ = fp8_fake_quantize(w, torch.tensor([2.0]), 8, 3)
        ep = torch.stack((torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)), 1).to(DEV).contiguous()
        return dense_conv2d_fused(x, wq, C, (s, s), (p, p), qin=(torch.tensor([6.0], device=DEV), 8, 3, 1),
                                  rq=(torch.tensor([40.0], device=DEV), 8, 3, 1), bn=(ep, 1, 0.0, 6.0))[0]

    old = _lib.set_option("dw3", form)
    try:
        g.manual_seed(1)
        y_new = run()
    finally:
        _lib.set_option("dw3", old)
    old = _lib.set_option("dw3", 0)
    try:
        g.manual_seed(1)
        y_old = run()
    finally:
        _lib.set_option("dw3", old)
    assert y_new.shape == y_old.shape
    assert torch.equal(torch.isnan(y_new), torch.isnan(y_old))
    fin = ~torch.isnan(y_old)
    assert torch.equal(y_new[fin], y_old[fin])


@pytest.mark.parametrize("shape", [(2, 3, 33, 33, 32, 3, 2, 1), (1, 3, 20, 17, 16, 3, 1, 1), (2, 2, 9, 9, 64, 4, 2, 0),
                                   (1, 32, 8, 8, 8, 1, 1, 0)], ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("fused", [False, True])
def test_small_conv_direct_form(shape, fused):
    """Small exact convolutions (K = Cin kh kw <= 32, Cout <= 64: the stem) on dn_direct_kernel (option
    "dn_direct" = 1) against the bf16 matrix-core form (0) and the float64 product: fp32 FMAs in k
    order, so within a few ulps of the matrix core's sum; with the config-1 tail (weight / input
    quantizers, rq, BN, clamp) fused, the quantizers' biases identical."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_conv2d, dense_conv2d_fused, dense_format
    Bn, C, H, W, Co, k, s, p = shape
    g = torch.Generator().manual_seed(Bn * C + H + Co + k)
    x = (torch.randn(Bn, C, H, W, generator=g) * 2).to(DEV)
    w = (torch.randn(Co, C, k, k, generator=g) * 0.3).to(DEV)

    def run():
        if not fused:
            return dense_conv2d(x, w.bfloat16().float(), dense_format(3), (s, s), (p, p)), None
        ep = torch.stack((torch.rand(Co, generator=g) + 0.5, torch.randn(Co, generator=g)), 1).to(DEV).contiguous()
        return dense_conv2d_fused(x, w, 1, (s, s), (p, p), qin=(torch.tensor([6.0], device=DEV), 8, 3, 1),
                                  rq=(torch.tensor([40.0], device=DEV), 8, 3, 1), bn=(ep, 1, 0.0, 6.0),
                                  wq=(torch.rand(Co, generator=g).to(DEV) + 0.2, 8, 3, 1))

    old = _lib.set_option("dn_direct", 1)
    try:
        g.manual_seed(3)
        y1, b1 = run()
        _lib.set_option("dn_direct", 0)
        g.manual_seed(3)
        y0, b0 = run()
    finally:
        _lib.set_option("dn_direct", old)
    if fused:
        assert all(torch.equal(b1[key], b0[key]) for key in b0)
        d = (y1 - y0).abs()
        # (the fused rq rounds to the FP8 grid: a last-bit sum difference can move a value one step)
        assert (d == 0).float().mean() > 0.995
    else:
        ref = torch.nn.functional.conv2d(x.double(), w.bfloat16().double(), stride=s, padding=p)
        assert torch.allclose(y1.double(), ref, rtol=1e-5, atol=1e-4)
        assert torch.allclose(y1, y0, rtol=1e-5, atol=1e-5)
