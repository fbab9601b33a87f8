"""The E4M3 tensor-bias (depthwise) table kernel conv_tbx_kernel (csrc/conv_tbx.h).

Single-output-channel groups take the reference's tensor-bias semantics.  For E4M3,
s2n, qbma, a {0,1} or zero table, 3-wide kernel rows and stride 1 / 2 the term is a table value
times the operands' binades plus the expo-0-binade and F7 fix-ups.  Checked here:
  * every one of the 256 x 256 E4M3 code pairs as a term, bit-exact against the oracle's
    tensor-bias terms: a 3x3 depthwise conv whose weights are zero except one tap makes every
    output exactly one term (several bias triples, both tables, the expo-0 binade and the F7
    band included: biases put products near 2^-bR);
  * sums of realistic MobileNetV2-like depthwise layers (stride 1 and 2, 3x3) within the bar;
  * an off-grid input raises the gate and the exact kernel's result is returned.
The launch's gate word is read back: 0 proves the table form produced the result.  E5M2 (round 4:
the same form with 2-bit mantissas; the zero table of zero_table_ext and a {0,1} table): every code
pair and layer sums likewise.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
E, M = 4, 3


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _codes(bias):
    e = np.repeat(np.arange(16), 8)
    m = np.tile(np.arange(8), 16)
    v = np.where(e == 0, np.ldexp(m / 8.0, 1 - bias), np.ldexp(1.0 + m / 8.0, e - bias))
    return np.concatenate([v, -v]).astype(np.float32)


def _dw_raw(x, w, bA, bW, bR, table, flags, stride, pad, fmt=(E, M)):
    """fp8a_conv2d on a depthwise layer with a caller-owned workspace: (y, gate word)."""
    from fp8_quantization_amd import _lib
    L = _lib.load()
    Bn, C, H, W = x.shape
    kh, kw = w.shape[2], w.shape[3]
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    xt = torch.as_tensor(np.ascontiguousarray(x)).to(DEV)
    wt = torch.as_tensor(np.ascontiguousarray(w)).to(DEV)
    y = torch.empty((Bn, C, Ho, Wo), dtype=torch.float32, device=DEV)
    n = int(L.fp8a_conv2d_workspace_size(Bn, C, H, W, C, kh, kw, stride, stride, pad, pad, 1, 1, C))
    ws = torch.zeros(n, dtype=torch.uint8, device=DEV)
    tA = torch.tensor([bA], dtype=torch.int32, device=DEV)
    tW = torch.as_tensor(np.asarray(bW, np.int32)).to(DEV)
    tR = torch.tensor([bR], dtype=torch.int32, device=DEV)
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32))
    rc = L.fp8a_conv2d(_lib.dev_ptr(xt), _lib.dev_ptr(wt), _lib.dev_ptr(y), Bn, C, H, W, C, kh, kw, stride, stride,
                       pad, pad, 1, 1, C, fmt[0], fmt[1], _lib.dev_ptr(tA), _lib.dev_ptr(tW), _lib.dev_ptr(tR),
                       _lib.host_ptr(tab), flags, _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_conv2d")
    torch.cuda.synchronize()
    return y.cpu().numpy(), int(ws[:4].view(torch.int32).item())


def _terms_equal(got, ref, what):
    same = (got.view(np.uint32) == ref.view(np.uint32)) | ((got == 0) & (ref == 0))
    if not same.all():
        i = tuple(np.argwhere(~same)[0])
        raise AssertionError(f"{what}: {np.count_nonzero(~same)} terms differ; first at {i}: "
                             f"got {got[i]!r} ref {ref[i]!r}")


FL = orc.flags_of(approx=True, s2n=True, qbma=True)


@pytest.mark.parametrize("table", ["nocomp", "comp"])
@pytest.mark.parametrize("biases", [(12, 12, 8), (10, 13, 7), (9, 9, 2), (14, 14, 20), (8, 8, 3)])
@pytest.mark.parametrize("stride", [1, 2])
def test_every_code_pair_bitexact(biases, table, stride):
    bA, bW_, bR = biases
    a = _codes(bA)          # 256 input values: one image of 16 x 16 pixels, same in every channel
    b = _codes(bW_)         # 256 channels, channel c's weight = b[c] at the center tap
    C = 256
    if stride == 1:
        x = np.broadcast_to(a.reshape(1, 1, 16, 16), (1, C, 16, 16)).copy()
        pad = 1
    else:  # stride 2 with padding 1: output (i, j) centres on input (2i, 2j)
        x = np.zeros((1, C, 32, 32), np.float32)
        x[:, :, 0::2, 0::2] = a.reshape(1, 1, 16, 16)
        pad = 1
    w = np.zeros((C, 1, 3, 3), np.float32)
    w[:, 0, 1, 1] = b
    bW = np.full(C, bW_, np.int32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_comp" if table == "comp" else "E4M3_table_nocomp"]
    y, gate = _dw_raw(x, w, bA, bW, bR, tab, FL, stride, pad)
    assert gate == 0, "gate raised: the table form did not produce these terms"
    ref = orc.terms(a.reshape(-1, 1), b.reshape(1, -1), E, M, bA, bW, bR, tab, FL | orc.TB)[:, 0, :]  # [256 a, 256 b]
    got = y[0].reshape(C, 256).T  # [pixel = a index, channel = b index]
    _terms_equal(got, ref, f"biases {biases} {table} stride {stride}")


def _grid(rng, shape, bias, zero_frac=0.0, lo=3):
    expo = rng.integers(lo, 16, size=shape)
    mant = rng.integers(0, 8, size=shape)
    v = np.ldexp(1.0 + mant / 8.0, expo - bias) * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


@pytest.mark.parametrize("cfg", [dict(C=32, hw=28, s=1), dict(C=24, hw=29, s=2), dict(C=48, hw=7, s=1),
                                 dict(C=16, hw=14, s=2)])
def test_depthwise_layer_sums(cfg):
    rng = np.random.default_rng(cfg["C"] * 100 + cfg["hw"])
    bA, bR = 10, 9
    C, hw, s = cfg["C"], cfg["hw"], cfg["s"]
    x = _grid(rng, (3, C, hw, hw), bA, zero_frac=0.4)
    bW = rng.integers(12, 16, size=C).astype(np.int32)
    w = _grid(rng, (C, 1, 3, 3), bW[:, None, None, None])
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    y, gate = _dw_raw(x, w, bA, bW, bR, tab, FL, s, 1)
    assert gate == 0
    cols = torch.nn.functional.unfold(torch.from_numpy(x), (3, 3), padding=1, stride=s)
    cols = cols.transpose(1, 2).reshape(-1, C * 9).numpy()
    for c in range(C):
        ref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, bA, bW[c:c + 1], bR, tab,
                            FL | orc.TB, with_abs=True)
        got = y[:, c].reshape(-1, 1).astype(np.float64)
        assert np.all(np.abs(got - ref) <= gio.sum_tolerance(S.astype(np.float64))), f"channel {c}"


def test_off_grid_input_falls_back():
    rng = np.random.default_rng(4)
    bA, bR = 10, 9
    x = _grid(rng, (2, 8, 9, 9), bA, zero_frac=0.3)
    x[1, 2, 4, 4] = 0.3
    bW = np.full(8, 13, np.int32)
    w = _grid(rng, (8, 1, 3, 3), 13)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    y, gate = _dw_raw(x, w, bA, bW, bR, tab, FL, 1, 1)
    assert gate != 0
    cols = torch.nn.functional.unfold(torch.from_numpy(x), (3, 3), padding=1).transpose(1, 2).reshape(-1, 72).numpy()
    for c in range(8):
        ref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, bA, bW[c:c + 1], bR, tab,
                            FL | orc.TB, with_abs=True)
        got = y[:, c].reshape(-1, 1).astype(np.float64)
        assert np.all(np.abs(got - ref) <= gio.sum_tolerance(S.astype(np.float64))), f"channel {c}"


# ---------------------------------------------------------------------------------------- E5M2
def _codes_e5m2(bias):
    e = np.repeat(np.arange(32), 4)
    m = np.tile(np.arange(4), 32)
    v = np.where(e == 0, np.ldexp(m / 4.0, 1 - bias), np.ldexp(1.0 + m / 4.0, e - bias))
    return np.concatenate([v, -v]).astype(np.float32)


def _table_e5m2(kind):
    if kind == "zero":
        return gio.load("g2_matmul.npz")["E5M2_table_zero"]
    return np.array([[0, 1, 0, 1], [1, 0, 1, 0], [0, 0, 1, 1], [1, 1, 0, 0]], np.int32)


@pytest.mark.parametrize("table", ["zero", "w1"])
@pytest.mark.parametrize("biases", [(20, 20, 9), (16, 24, 12), (12, 12, 2), (28, 28, 40), (24, 20, 30)])
@pytest.mark.parametrize("stride", [1, 2])
def test_e5m2_every_code_pair_bitexact(biases, table, stride):
    bA, bW_, bR = biases
    a, b = _codes_e5m2(bA), _codes_e5m2(bW_)
    C = 256
    if stride == 1:
        x = np.broadcast_to(a.reshape(1, 1, 16, 16), (1, C, 16, 16)).copy()
    else:
        x = np.zeros((1, C, 32, 32), np.float32)
        x[:, :, 0::2, 0::2] = a.reshape(1, 1, 16, 16)
    w = np.zeros((C, 1, 3, 3), np.float32)
    w[:, 0, 1, 1] = b
    bW = np.full(C, bW_, np.int32)
    tab = _table_e5m2(table)
    y, gate = _dw_raw(x, w, bA, bW, bR, tab, FL, stride, 1, fmt=(5, 2))
    ref = orc.terms(a.reshape(-1, 1), b.reshape(1, -1), 5, 2, bA, bW, bR, tab, FL | orc.TB)[:, 0, :]
    assert gate == 0, "gate raised: the table form did not produce these terms"
    got = y[0].reshape(C, 256).T
    _terms_equal(got, ref, f"E5M2 biases {biases} {table} stride {stride}")


@pytest.mark.parametrize("cfg", [dict(C=32, hw=28, s=1), dict(C=24, hw=29, s=2), dict(C=16, hw=14, s=2)])
def test_e5m2_depthwise_layer_sums(cfg):
    rng = np.random.default_rng(cfg["C"] * 7 + cfg["hw"])
    bA, bR = 18, 16
    C, hw, s = cfg["C"], cfg["hw"], cfg["s"]
    expo = rng.integers(6, 32, size=(3, C, hw, hw))
    x = np.ldexp(1.0 + rng.integers(0, 4, size=expo.shape) / 4.0, expo - bA) * rng.choice([-1.0, 1.0], size=expo.shape)
    x[rng.random(x.shape) < 0.4] = 0.0
    x = x.astype(np.float32)
    bW = rng.integers(20, 24, size=C).astype(np.int32)
    we = rng.integers(6, 32, size=(C, 1, 3, 3))
    w = (np.ldexp(1.0 + rng.integers(0, 4, size=we.shape) / 4.0, we - bW[:, None, None, None])
         * rng.choice([-1.0, 1.0], size=we.shape)).astype(np.float32)
    tab = _table_e5m2("zero")
    y, gate = _dw_raw(x, w, bA, bW, bR, tab, FL, s, 1, fmt=(5, 2))
    assert gate == 0
    cols = torch.nn.functional.unfold(torch.from_numpy(x), (3, 3), padding=1, stride=s)
    cols = cols.transpose(1, 2).reshape(-1, C * 9).numpy()
    for c in range(C):
        ref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), 5, 2, bA, bW[c:c + 1], bR, tab,
                            FL | orc.TB, with_abs=True)
        got = y[:, c].reshape(-1, 1).astype(np.float64)
        assert np.all(np.abs(got - ref) <= gio.sum_tolerance(S.astype(np.float64))), f"channel {c}"


@pytest.mark.parametrize("fmt", [(4, 3), (5, 2)], ids=["E4M3", "E5M2"])
@pytest.mark.parametrize("cfg", [dict(C=16, hw=15, s=1), dict(C=24, hw=13, s=2), dict(C=8, hw=1, s=1),
                                 dict(C=8, hw=6, s=2), dict(C=32, hw=112, s=1), dict(C=12, hw=56, s=2),
                                 dict(C=40, hw=7, s=1), dict(C=20, hw=14, s=2)])
def test_two_row_and_staged_forms_bit_identical(fmt, cfg):
    """The depthwise table form's three kernels on the same layer: conv_tbx_kernel with option
    "tbx_rw" = 1 and 2 (two output rows per thread) after the word pre-pass, and the LDS-staged
    conv_tbs_kernel (option "tbs", the default: pre-pass fused, bands of rows of one plane or groups
    of whole planes) -- the same terms in the same (ky, kx) order per output, so bit-identical
    outputs (odd Ho, 1-pixel planes, ragged quads, MobileNetV2's 112 / 56 / 14 / 7 planes)."""
    from fp8_quantization_amd import _lib
    rng = np.random.default_rng(cfg["C"] + cfg["hw"] + cfg["s"])
    E_, M_ = fmt
    C, hw, s = cfg["C"], cfg["hw"], cfg["s"]
    if fmt == (4, 3):
        bA, bR = 10, 9
        x = _grid(rng, (2, C, hw, hw), bA, zero_frac=0.3)
        bW = rng.integers(12, 16, size=C).astype(np.int32)
        w = _grid(rng, (C, 1, 3, 3), bW[:, None, None, None])
        tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    else:
        bA, bR = 18, 16
        x = (np.ldexp(1.0 + rng.integers(0, 4, size=(2, C, hw, hw)) / 4.0, rng.integers(-12, 14, size=(2, C, hw, hw)))
             * rng.choice([-1.0, 1.0], size=(2, C, hw, hw))).astype(np.float32)
        bW = rng.integers(20, 24, size=C).astype(np.int32)
        w = (np.ldexp(1.0 + rng.integers(0, 4, size=(C, 1, 3, 3)) / 4.0, rng.integers(-14, 8, size=(C, 1, 3, 3)))
             * rng.choice([-1.0, 1.0], size=(C, 1, 3, 3))).astype(np.float32)
        tab = _table_e5m2("zero")
    old, old_tbs = _lib.set_option("tbx_rw", 1), _lib.set_option("tbs", 0)
    try:
        y1, g1 = _dw_raw(x, w, bA, bW, bR, tab, FL, s, 1, fmt=fmt)
        _lib.set_option("tbx_rw", 2)
        y2, g2 = _dw_raw(x, w, bA, bW, bR, tab, FL, s, 1, fmt=fmt)
        _lib.set_option("tbs", 1)
        y3, g3 = _dw_raw(x, w, bA, bW, bR, tab, FL, s, 1, fmt=fmt)
        _lib.set_option("tbs", 2)  # the LDS-DMA-staged conv_tbsg_kernel
        y4, g4 = _dw_raw(x, w, bA, bW, bR, tab, FL, s, 1, fmt=fmt)
    finally:
        _lib.set_option("tbx_rw", old)
        _lib.set_option("tbs", old_tbs)
    assert g1 == 0 and g2 == 0 and g3 == 0 and g4 == 0
    assert np.array_equal(y1.view(np.uint32), y2.view(np.uint32))
    assert np.array_equal(y1.view(np.uint32), y3.view(np.uint32))
    assert np.array_equal(y1.view(np.uint32), y4.view(np.uint32))


@pytest.mark.parametrize("fmt", [(4, 3), (5, 2)], ids=["E4M3", "E5M2"])
def test_staged_form_full_model_bit_identical(fmt):
    """A full-size MobileNetV2 (224 x 224, width 1: every depthwise geometry of the benchmark) in
    the fixed-range state: logits with the staged depthwise form (input quantizer and BN epilogue
    fused into it) equal those of the pre-pass + gather form to the bit."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
    torch.manual_seed(5)
    m = mobilenet_v2_approx(input_size=224, n_class=1000, bn_stats_batches=1, device=DEV, withComp=False,
                            expo_width=fmt[0], mant_width=fmt[1]).to(DEV).eval()
    g = torch.Generator().manual_seed(2)
    m.quantized()
    m.estimate_ranges()
    with torch.no_grad():
        m(torch.randn((2, 3, 224, 224), generator=g).to(DEV))
    m.fix_ranges()
    x = torch.randn((2, 3, 224, 224), generator=g).to(DEV)
    with torch.no_grad():
        y1 = m(x).cpu().numpy()
    old = _lib.set_option("tbs", 0)
    try:
        with torch.no_grad():
            y0 = m(x).cpu().numpy()
        _lib.set_option("tbs", 2 if old != 2 else 1)  # the other staged form
        with torch.no_grad():
            y2 = m(x).cpu().numpy()
    finally:
        _lib.set_option("tbs", old)
    assert np.isfinite(y1).all()
    assert np.array_equal(y0.view(np.uint32), y1.view(np.uint32))
    assert np.array_equal(y0.view(np.uint32), y2.view(np.uint32))


def test_gate_arena_is_clean_after_a_fallback():
    """The depthwise gate word is the stream's flag arena (fp8approx.hip: flag_arena), left zero by
    the gated direct kernel: a flagged launch, then a clean one reports gate 0 and runs no
    fallback launch, then a flagged one again reports its gate."""
    from fp8_quantization_amd import _lib
    rng = np.random.default_rng(5)
    bA, bR = 10, 9
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    xb = _grid(rng, (2, 8, 9, 9), bA, zero_frac=0.3)
    xb[1, 2, 4, 4] = 0.3
    bW = np.full(8, 13, np.int32)
    w = _grid(rng, (8, 1, 3, 3), 13)
    xg = _grid(rng, (2, 8, 9, 9), bA, zero_frac=0.3)
    cols = torch.nn.functional.unfold(torch.from_numpy(xg), (3, 3), padding=1).transpose(1, 2).reshape(-1, 72).numpy()
    for _ in range(2):
        _, gate = _dw_raw(xb, w, bA, bW, bR, tab, FL, 1, 1)
        assert gate != 0
        _lib.fallback_stats(reset=True)
        y, gate = _dw_raw(xg, w, bA, bW, bR, tab, FL, 1, 1)
        assert gate == 0 and _lib.fallback_stats()["tb_launches"] == 0
        for c in range(8):
            ref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, bA, bW[c:c + 1], bR, tab,
                                FL | orc.TB, with_abs=True)
            got = y[:, c].reshape(-1, 1).astype(np.float64)
            assert np.all(np.abs(got - ref) <= gio.sum_tolerance(S.astype(np.float64))), f"channel {c}"
