"""GPU parity of the v5 integer-adder model (approx_matmul_whole_v5.py)
against the reference's own values (tests/golden/g7_v5.npz) and the CPU oracle.

Bars: every per-product term bit-exact (terms kernel, and the fast tiled kernel through
K = 1 launches); sums within 1e-5 x sum|terms| (order differs)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu

META = gio.meta()
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def t(x, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(x)).to(device=DEV, dtype=dtype)


def same_bits(got, ref):
    got, ref = np.asarray(got, np.float32), np.asarray(ref, np.float32)
    return (got.view(np.uint32) == ref.view(np.uint32)) | ((got == 0) & (ref == 0))


@pytest.mark.parametrize("case", META["g7"], ids=lambda c: c["key"])
def test_g7_v5_terms_and_sums(case):
    import fp8_quantization_amd.approx_v5 as v5
    from fp8_quantization_amd.approx_ops import approx_terms, make_flags_v5
    g = gio.load("g7_v5.npz")
    A, B, tab, fl = gio.v5_case(case)
    E, M, b = case["E"], case["M"], case["bias"]
    sw = dict(sim_hw_add_OFUF=case["ofuf"], with_OF_opt=case["of_opt"], with_UF_opt=case["uf_opt"])
    Tref = g[case["key"] + "_T"]
    # exact (terms) kernel
    T = approx_terms(t(A[:6]), t(B[:, :6]), E, M, b, b, b, torch.as_tensor(tab),
                     flags=make_flags_v5(**sw)).cpu().numpy()
    assert same_bits(T, Tref).all(), "terms kernel"
    # fast tiled kernel, one product per launch (K = 1)
    for k in range(A.shape[1]):
        c = v5.custom_matmul_vectorize(t(A[:6, k:k + 1]), t(B[k:k + 1, :6]), E, M,
                                       None if case["default_bias"] else b, torch.as_tensor(tab), **sw).cpu().numpy()
        assert same_bits(c, Tref[:, k, :]).all(), f"fast kernel term k={k}"
    # sums (v5 signature; None = the default bias, as in the reference)
    C = v5.custom_matmul_vectorize(t(A), t(B), E, M, None if case["default_bias"] else b, torch.as_tensor(tab),
                                   **sw).cpu().numpy()
    _, S = orc.matmul(A, B, E, M, b, b, b, tab, fl, with_abs=True)
    assert np.all(np.abs(C.astype(np.float64) - g[case["key"] + "_C"]) <= gio.sum_tolerance(S))


@pytest.mark.parametrize("groups,cout", [(1, 24), (4, 8), (8, 8)])
def test_v5_conv2d_per_operand_biases(groups, cout):
    """Implicit-GEMM conv in v5 mode with per-operand / per-channel biases (the operator-level
    generalisation), incl. single-output-channel groups, vs the oracle on unfolded inputs."""
    from fp8_quantization_amd.approx_v5 import approx_conv2d_v5, get_comp_table_NN
    rng = np.random.default_rng(groups * 100 + cout)
    E, M, bA, bR = 3, 4, 4, 5
    cin, hw, k = 8, 9, 3
    x = np.ldexp(rng.integers(16, 32, size=(2, cin, hw, hw)) / 16.0, rng.integers(-5, 3, size=(2, cin, hw, hw)))
    x[rng.random(x.shape) < 0.3] = 0.0
    x = (x * rng.choice([-1.0, 1.0], size=x.shape)).astype(np.float32)
    cig = cin // groups
    w = np.ldexp(rng.integers(16, 32, size=(cout, cig, k, k)) / 16.0, rng.integers(-8, 0, size=(cout, cig, k, k)))
    w = (w * rng.choice([-1.0, 1.0], size=w.shape)).astype(np.float32)
    bW = rng.integers(5, 8, size=cout).astype(np.int32)
    tab = get_comp_table_NN(E, M, True, 4)
    for sw in [dict(), dict(sim_hw_add_OFUF=True, with_OF_opt=True, with_UF_opt=True)]:
        y = approx_conv2d_v5(t(x), t(w), E, M, bA, t(bW, torch.int32), bR, tab, padding=(1, 1), groups=groups,
                             **sw).cpu().numpy()
        cols = torch.nn.functional.unfold(torch.from_numpy(x), (k, k), padding=1).transpose(1, 2)
        cols = cols.reshape(-1, cols.shape[2]).numpy()
        cog, Kg = cout // groups, cig * k * k
        fl = orc.flags_v5(sw.get("sim_hw_add_OFUF", False), sw.get("with_OF_opt", False), sw.get("with_UF_opt", False))
        for gi in range(groups):
            Wg = w[gi * cog:(gi + 1) * cog].reshape(cog, -1).T
            Cref, S = orc.matmul(cols[:, gi * Kg:(gi + 1) * Kg], Wg, E, M, bA, bW[gi * cog:(gi + 1) * cog], bR,
                                 tab.numpy(), fl, with_abs=True)
            got = y[:, gi * cog:(gi + 1) * cog].transpose(0, 2, 3, 1).reshape(-1, cog)
            assert np.all(np.abs(got.astype(np.float64) - Cref) <= gio.sum_tolerance(S)), f"group {gi} {sw}"


def test_v5_operator_opt_in():
    """custom_approx_params["approx_version"] = 5 routes QCustomBNConv2dTorch's approx product
    through the v5 kernel with the operator's own biases."""
    from fp8_quantization_amd.approx_v5 import approx_conv2d_v5, get_comp_table_NN
    from fp8_quantization_amd.resnet_workload import _conv, approx_qparams
    qp = approx_qparams(expo_width=3, mant_width=4, withComp=True)
    qp["custom_approx_params"].update(approx_version=5, sim_hw_add_OFUF=True, with_UF_opt=True)
    torch.manual_seed(3)
    m = _conv(qp, 16, 32, 3, 1, 1, True).to(DEV).eval()
    x = torch.randn(2, 16, 10, 10, device=DEV).relu()
    with torch.no_grad():
        m.quantized()
        m.estimate_ranges()
        m(x)
        m.fix_ranges()
        xq = m.activation_quantizer(x)
        wq, _ = m.get_params()
        got = m.run_forward(xq, wq, None)
        ref = approx_conv2d_v5(xq, wq, 3, 4, m.get_acts_fp_bias(), m.get_weights_fp_bias().reshape(-1),
                               m.get_res_fp_bias(), get_comp_table_NN(3, 4, True, 3), sim_hw_add_OFUF=True,
                               with_UF_opt=True, padding=(1, 1))
    assert torch.equal(got, ref)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("sw", [dict(sim_hw_add_OFUF=True), dict(sim_hw_add_OFUF=True, with_OF_opt=True, with_UF_opt=True),
                                dict(sim_hw_add_OFUF=True, with_UF_opt=True)], ids=["wrap", "wrap_of_uf", "wrap_uf"])
def test_v5_depthwise_e5m2_word_form(stride, sw):
    """MobileNetV2-like E5M2 depthwise layers in v5 mode with the adder wrap (BASELINE config 3's
    switches) run the word form conv_v5dw_kernel (a "fast" launch, no literal recompute); every
    output equals the oracle's sum of its 9 v5 terms within the bar, and single-tap outputs (the
    other 8 terms of a zero weight row pinned separately) are bit-exact terms."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_v5 import approx_conv2d_v5
    rng = np.random.default_rng(stride * 10 + len(sw))
    E, M, bA, bR = 5, 2, 16, 12
    C, hw = 24, 15
    x = np.ldexp(1.0 + rng.integers(0, 4, size=(2, C, hw, hw)) / 4.0, rng.integers(-14, 16, size=(2, C, hw, hw)))
    x[rng.random(x.shape) < 0.4] = 0.0
    x = (x * rng.choice([-1.0, 1.0], size=x.shape)).astype(np.float32)
    w = np.ldexp(1.0 + rng.integers(0, 4, size=(C, 1, 3, 3)) / 4.0, rng.integers(-12, 11, size=(C, 1, 3, 3)))
    w = (w * rng.choice([-1.0, 1.0], size=w.shape)).astype(np.float32)
    bW = rng.integers(14, 20, size=C).astype(np.int32)
    tab = torch.zeros(4, 4, dtype=torch.int32)  # the E5M2 zero table (zero_table_ext)
    _lib.path_stats(reset=True)
    _lib.fallback_stats(reset=True)
    y = approx_conv2d_v5(t(x), t(w), E, M, bA, t(bW, torch.int32), bR, tab, stride=(stride, stride), padding=(1, 1),
                         groups=C, **sw).cpu().numpy()
    paths = _lib.path_stats(reset=True)
    assert paths["fast"] == 1 and paths["exact"] == 0, paths
    assert _lib.fallback_stats(reset=True)["tb_launches"] == 0
    cols = torch.nn.functional.unfold(torch.from_numpy(x), (3, 3), padding=1, stride=stride).transpose(1, 2)
    cols = cols.reshape(-1, C * 9).numpy()
    fl = orc.flags_v5(True, sw.get("with_OF_opt", False), sw.get("with_UF_opt", False))
    for c in range(C):
        ref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, bA, bW[c:c + 1], bR, tab.numpy(), fl,
                            with_abs=True)
        got = y[:, c].reshape(-1, 1).astype(np.float64)
        assert np.all(np.abs(got - ref) <= gio.sum_tolerance(S)), f"channel {c}"
        tm = orc.terms(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, bA, bW[c:c + 1], bR, tab.numpy(), fl)
        seq = np.zeros(tm.shape[0], np.float32)
        for k in range(9):
            seq = (seq + tm[:, k, 0].astype(np.float32)).astype(np.float32)
        assert same_bits(y[:, c].reshape(-1), seq).all(), f"channel {c}: not the literal k-order sum"


V5DS_SHAPES = [  # (Bn, C, H, W, stride): MobileNetV2 geometries (whole planes and row bands), ragged ones
    (2, 32, 112, 112, 1), (2, 96, 112, 112, 2), (2, 144, 56, 56, 2), (3, 192, 28, 28, 1), (4, 576, 14, 14, 2),
    (5, 960, 7, 7, 1), (1, 3, 5, 9, 1), (2, 5, 13, 7, 2), (1, 4, 9, 300, 1), (1, 2, 1, 1, 1)]


@pytest.mark.parametrize("shape", V5DS_SHAPES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("qin", [False, True])
def test_v5_depthwise_staged_form_bit_identical(shape, qin):
    """The staged v5 depthwise kernel (conv_v5ds_kernel, option "v5ds" = 1: LDS-DMA window, both word
    pre-passes fused, 4 outputs per thread) against the pre-pass + conv_v5dw_kernel form (v5ds = 0):
    the same bits, with and without the fused input quantizer and its bias."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import approx_conv2d
    Bn, C, H, W, s = shape
    rng = np.random.default_rng(Bn * C + H * W + s + int(qin))
    x = np.ldexp(1.0 + rng.integers(0, 4, size=(Bn, C, H, W)) / 4.0, rng.integers(-14, 6, size=(Bn, C, H, W)))
    x[rng.random(x.shape) < 0.3] = 0.0
    x = (x * rng.choice([-1.0, 1.0], size=x.shape)).astype(np.float32)
    if qin:
        x = x * np.float32(1.37)  # off the grid: the fused quantizer rounds it
    w = np.ldexp(1.0 + rng.integers(0, 4, size=(C, 1, 3, 3)) / 4.0, rng.integers(-12, 4, size=(C, 1, 3, 3)))
    w = (w * rng.choice([-1.0, 1.0], size=w.shape)).astype(np.float32)
    bW = t(rng.integers(14, 20, size=C).astype(np.int32), torch.int32)
    bR = torch.tensor([12], dtype=torch.int32, device=DEV)
    tab = torch.as_tensor(np.array([[0, -1, 2, 0], [1, 0, -2, 1], [0, 3, 0, -1], [-3, 1, 1, 0]], np.int32))
    fl = orc.flags_v5(True, True, True)
    kw = dict(flags=fl, stride=(s, s), padding=(1, 1), groups=C)
    bA = None if qin else torch.tensor([16], dtype=torch.int32, device=DEV)
    q = (torch.tensor([20.0], device=DEV), 8, 2, 1) if qin else None

    def run():
        r = approx_conv2d(t(x), t(w), 5, 2, bA, bW, bR, tab, qin=q, **kw)
        return (r[0], r[1]) if qin else (r, None)

    old = _lib.set_option("v5ds", 1)
    try:
        y1, b1 = run()
        _lib.set_option("v5ds", 0)
        y0, b0 = run()
    finally:
        _lib.set_option("v5ds", old)
    assert torch.equal(y1.view(torch.int32), y0.view(torch.int32))
    if qin:
        assert torch.equal(b1, b0)


def _e5m2_codes(bias):
    e = np.repeat(np.arange(32), 4)
    m = np.tile(np.arange(4), 32)
    v = np.where(e == 0, np.ldexp(m / 4.0, 1 - bias), np.ldexp(1.0 + m / 4.0, e - bias))
    return np.concatenate([v, -v]).astype(np.float32)


def _v5_e5m2_tables():
    # (v5 has no compensation table for E5M2: approx_matmul_whole_v5.py:540 raises, so the
    # reference-table case is the zero table; "signed" exercises the table path's arithmetic)
    return {"zero": np.zeros((4, 4), np.int32),
            "signed": np.array([[0, -1, 2, 0], [1, 0, -2, 1], [0, 3, 0, -1], [-3, 1, 1, 0]], np.int32)}


SWITCHES = [dict(sim_hw_add_OFUF=True), dict(sim_hw_add_OFUF=True, with_UF_opt=True),
            dict(sim_hw_add_OFUF=True, with_OF_opt=True), dict(sim_hw_add_OFUF=True, with_OF_opt=True, with_UF_opt=True)]
SW_IDS = ["wrap", "wrap_uf", "wrap_of", "wrap_of_uf"]


@pytest.mark.parametrize("sw", SWITCHES, ids=SW_IDS)
@pytest.mark.parametrize("biases", [(16, 16, 12), (12, 20, 30), (20, 10, 2), (8, 8, -20)])
@pytest.mark.parametrize("table", ["zero", "signed"])
def test_v5mx_every_code_pair_bitexact(sw, biases, table):
    """gemm_v5mx_kernel (E5M2, the adder wrap on): every one of the 256 x 256 code pairs as a
    K = 1 product equals the oracle's v5 term bit for bit, for each OF / UF switch pair (the
    ragged last K-tile masks the seven padded K-steps)."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_v5 import approx_matmul_v5
    tab = _v5_e5m2_tables()[table]
    bA, bB, bR = biases
    A = _e5m2_codes(bA).reshape(-1, 1)
    B = _e5m2_codes(bB).reshape(1, -1)
    _lib.path_stats(reset=True)
    C = approx_matmul_v5(t(A), t(B), 5, 2, bA, bB, bR, torch.as_tensor(tab), **sw).cpu().numpy()
    paths = _lib.path_stats(reset=True)
    assert paths["v5mx"] == 1, paths
    fl = orc.flags_v5(True, sw.get("with_OF_opt", False), sw.get("with_UF_opt", False))
    ref = orc.terms(A, B, 5, 2, bA, bB, bR, tab, fl)[:, 0, :]
    ok = same_bits(C, ref)
    assert ok.all(), f"{np.count_nonzero(~ok)} terms differ; first {np.argwhere(~ok)[0]}"


@pytest.mark.parametrize("sw", SWITCHES, ids=SW_IDS)
@pytest.mark.parametrize("shape", [(300, 200, 72), (64, 37, 16), (1000, 960, 32)])
def test_v5mx_sums_within_bar(sw, shape):
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_v5 import approx_matmul_v5
    Mr, K, N = shape
    rng = np.random.default_rng(Mr + K + N + len(sw))
    bA, bR = 16, 14
    A = np.ldexp(1.0 + rng.integers(0, 4, size=(Mr, K)) / 4.0, rng.integers(-16, 16, size=(Mr, K)))
    A[rng.random(A.shape) < 0.3] = 0.0
    A = (A * rng.choice([-1.0, 1.0], size=A.shape)).astype(np.float32)
    B = (np.ldexp(1.0 + rng.integers(0, 4, size=(K, N)) / 4.0, rng.integers(-14, 8, size=(K, N)))
         * rng.choice([-1.0, 1.0], size=(K, N))).astype(np.float32)
    bB = rng.integers(14, 19, size=N).astype(np.int32)
    tab = _v5_e5m2_tables()["signed"]
    _lib.path_stats(reset=True)
    C = approx_matmul_v5(t(A), t(B), 5, 2, bA, t(bB, torch.int32), bR, torch.as_tensor(tab), **sw).cpu().numpy()
    assert _lib.path_stats(reset=True)["v5mx"] == 1
    fl = orc.flags_v5(True, sw.get("with_OF_opt", False), sw.get("with_UF_opt", False))
    ref, S = orc.matmul(A, B, 5, 2, bA, bB, bR, tab, fl, with_abs=True)
    assert np.all(np.abs(C.astype(np.float64) - ref) <= gio.sum_tolerance(S))


@pytest.mark.parametrize("k,pad,stride", [(3, 1, 1), (3, 1, 2), (1, 0, 1)])
def test_v5mx_conv2d_e5m2(k, pad, stride):
    """The implicit-GEMM conv on gemm_v5mx_kernel: the zero border of the word image gives the
    padded positions the v5 term of a zero operand, as the reference's im2col does."""
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_v5 import approx_conv2d_v5
    rng = np.random.default_rng(k * 10 + stride)
    E, M, bA, bR = 5, 2, 16, 12
    cin, cout, hw = 24, 40, 11
    x = np.ldexp(1.0 + rng.integers(0, 4, size=(2, cin, hw, hw)) / 4.0, rng.integers(-14, 14, size=(2, cin, hw, hw)))
    x[rng.random(x.shape) < 0.4] = 0.0
    x = (x * rng.choice([-1.0, 1.0], size=x.shape)).astype(np.float32)
    w = (np.ldexp(1.0 + rng.integers(0, 4, size=(cout, cin, k, k)) / 4.0, rng.integers(-12, 6, size=(cout, cin, k, k)))
         * rng.choice([-1.0, 1.0], size=(cout, cin, k, k))).astype(np.float32)
    bW = rng.integers(14, 20, size=cout).astype(np.int32)
    tab = _v5_e5m2_tables()["zero"]
    sw = dict(sim_hw_add_OFUF=True, with_OF_opt=True, with_UF_opt=True)
    _lib.path_stats(reset=True)
    y = approx_conv2d_v5(t(x), t(w), E, M, bA, t(bW, torch.int32), bR, torch.as_tensor(tab), stride=(stride, stride),
                         padding=(pad, pad), **sw).cpu().numpy()
    assert _lib.path_stats(reset=True)["v5mx"] == 1
    cols = torch.nn.functional.unfold(torch.from_numpy(x), (k, k), padding=pad, stride=stride).transpose(1, 2)
    cols = cols.reshape(-1, cols.shape[2]).numpy()
    fl = orc.flags_v5(True, True, True)
    ref, S = orc.matmul(cols, w.reshape(cout, -1).T, E, M, bA, bW, bR, tab, fl, with_abs=True)
    got = y.transpose(0, 2, 3, 1).reshape(-1, cout).astype(np.float64)
    assert np.all(np.abs(got - ref) <= gio.sum_tolerance(S))
