"""GPU parity of the HIP path against the reference's golden vectors and the CPU oracle.

Bars:
  * integer fields (expo / mant), Q_R values and every per-product term: bit-exact
    (zeros compared by value: the per-term fixtures are one-element torch sums, which turn
    -0.0 into +0.0);
  * fp32 sums: |c - c_oracle| <= 1e-5 * sum_k |term| (+1e-30), c_oracle accumulated in double.
"""
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
    import fp8_quantization_amd as fa  # noqa: F401
    from fp8_quantization_amd import _lib
    _lib.load()


def fa():
    import fp8_quantization_amd as m
    return m


def t(x, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(x)).to(device=DEV, dtype=dtype)


def assert_terms_equal(got, ref, msg=""):
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | ((got == 0) & (ref == 0))
    if not same.all():
        i = np.argwhere(~same)[0]
        raise AssertionError(f"{msg}: {np.count_nonzero(~same)} terms differ; first at {tuple(i)}: "
                             f"got {got[tuple(i)]!r} ref {ref[tuple(i)]!r}")


def assert_sums_close(got, ref, abs_sum, msg=""):
    got = np.asarray(got, np.float64)
    err = np.abs(got - ref)
    tol = gio.sum_tolerance(np.asarray(abs_sum, np.float64))
    if not np.all(err <= tol):
        r = np.max(err / (np.asarray(abs_sum) + 1e-30))
        raise AssertionError(f"{msg}: sum error {r:.3e} x sum|v| exceeds 1e-5")


def g2_table(fmt, tname):
    return gio.load("g2_matmul.npz")[f"{fmt}_table_{tname}"]


# ------------------------------------------------------------------------------ G1 codecs
@pytest.mark.parametrize("case", META["g1"], ids=lambda c: c["key"])
def test_decompose_and_quant_bitexact(case):
    g = gio.load("g1_decompose.npz")
    key, E, M, b = case["key"], case["E"], case["M"], case["b"]
    x = t(g[key + "_x"])
    for tb in (0, 1):
        bias = torch.tensor([b], dtype=torch.int32, device=DEV) if tb else b
        for clip in (0, 1):
            sfx = f"_tb{tb}_c{clip}"
            e, m = fa().float_to_fpany_absint_torch(x, E, M, bias, clip_OF=bool(clip))
            q = fa().quant_to_fp_any_vectorize_torch(x, E, M, bias, clip_OF=bool(clip))
            np.testing.assert_array_equal(e.cpu().numpy(), g[key + sfx + "_expo"], err_msg=key + sfx)
            np.testing.assert_array_equal(m.cpu().numpy(), g[key + sfx + "_mant"], err_msg=key + sfx)
            np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), g[key + sfx + "_q"].view(np.uint32),
                                          err_msg=key + sfx)


# ------------------------------------------------------------------------------ G2 matmul
def _g2(case):
    g = gio.load("g2_matmul.npz")
    return g, g[case["fmt"] + "_A"], g[case["fmt"] + "_B"], g2_table(case["fmt"], case["table"])


@pytest.mark.parametrize("case", META["g2"], ids=lambda c: c["key"])
def test_g2_terms_kernel_bitexact(case):
    g, A, B, tab = _g2(case)
    T = fa().approx_terms(t(A[:8, :64]), t(B[:64, :8]), case["E"], case["M"], case["bA"], case["bB"], case["bR"],
                          torch.as_tensor(tab), flags=gio.flags_from(case))
    assert_terms_equal(T.cpu().numpy(), g[case["key"] + "_T"], case["key"])


@pytest.mark.parametrize("case", META["g2"], ids=lambda c: c["key"])
def test_g2_fast_kernel_per_term_bitexact(case):
    """The tiled fast kernel run with K=1 returns single terms: bit-exact against the oracle."""
    g, A, B, tab = _g2(case)
    fl = gio.flags_from(case)
    n = A.shape[0]
    ref = orc.terms(A[:, :16], B[:16, :], case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl)
    for k in range(16):
        C = fa().approx_matmul(t(A[:, k:k + 1]), t(B[k:k + 1, :]), case["E"], case["M"], case["bA"], case["bB"],
                               case["bR"], torch.as_tensor(tab), flags=fl)
        assert_terms_equal(C.cpu().numpy(), ref[:, k, :], f"{case['key']} k={k}")
    assert n == A.shape[0]


@pytest.mark.parametrize("case", META["g2"], ids=lambda c: c["key"])
def test_g2_fast_kernel_sums(case):
    g, A, B, tab = _g2(case)
    fl = gio.flags_from(case)
    C = fa().approx_matmul(t(A), t(B), case["E"], case["M"], case["bA"], case["bB"], case["bR"],
                           torch.as_tensor(tab), flags=fl).cpu().numpy()
    Cref, S = orc.matmul(A, B, case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl, with_abs=True)
    assert_sums_close(C, Cref, S, case["key"])
    # and against the reference's own fp32 sums on its 64x64 crop
    assert_sums_close(C[:64, :64], g[case["key"] + "_C"], S[:64, :64], case["key"] + " vs reference")


def test_custom_matmul_vectorize_signature_and_weight_view():
    """Reference signature; B given as weight.t() (k-contiguous view) is consumed in place."""
    g = gio.load("g2_matmul.npz")
    c = next(c for c in META["g2"] if c["key"].startswith("E3M4_comp3_a1_s1_q1_g0"))
    A, B = g["E3M4_A"], g["E3M4_B"]
    W = t(B.T.copy())  # [N, K] weight layout
    out = fa().custom_matmul_vectorize(t(A), W.t(), 3, 4, 3, 5, 5, torch.as_tensor(g2_table("E3M4", "comp3")),
                                       with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    Cref, S = orc.matmul(A, B, 3, 4, 3, 5, 5, g2_table("E3M4", "comp3"), gio.flags_from(c), with_abs=True)
    assert_sums_close(out.cpu().numpy(), Cref, S)
    with pytest.raises(AssertionError):
        fa().custom_matmul_vectorize(t(A), t(B[:10]), 3, 4, 3, 5, 5, None)


# ------------------------------------------------------------------------------ G3 captured layer
@pytest.mark.parametrize("case", META["g3"], ids=lambda c: c["key"])
def test_g3_debug_params_layer(case):
    g = gio.load("g3_debug.npz")
    tab = g2_table("E3M4", case["table"])
    bB = t(g["bB"], torch.int32)
    C = fa().approx_matmul(t(g["A"]), t(g["B"]), 3, 4, int(g["bA"][0]), bB, int(g["bR"][0]), torch.as_tensor(tab),
                           flags=gio.flags_from(case)).cpu().numpy()
    Cref, S = orc.matmul(g["A"], g["B"], 3, 4, int(g["bA"][0]), g["bB"].astype(np.int32), int(g["bR"][0]), tab,
                         gio.flags_from(case), with_abs=True)
    assert_sums_close(C, Cref, S, case["key"])
    assert_sums_close(C, g[case["key"] + "_C"], S, case["key"] + " vs reference")


# ------------------------------------------------------------------------------ G4 tensor bias
@pytest.mark.parametrize("case", META["g4"], ids=lambda c: c["key"])
def test_g4_tensor_bias(case):
    g = gio.load("g4_tensorbias.npz")
    A, B = g[case["fmt"] + "_A"], g[case["fmt"] + "_B"]
    tab = g2_table(case["fmt"], case["table"])
    fl = gio.flags_from(case, tb=True)
    T = fa().approx_terms(t(A), t(B), case["E"], case["M"], case["bA"], case["bB"], case["bR"], torch.as_tensor(tab),
                          flags=fl)
    assert_terms_equal(T.cpu().numpy(), g[case["key"] + "_T"], case["key"])
    C = fa().approx_matmul(t(A), t(B), case["E"], case["M"], case["bA"], case["bB"], case["bR"],
                           torch.as_tensor(tab), flags=fl).cpu().numpy()
    Cref, S = orc.matmul(A, B, case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl, with_abs=True)
    assert_sums_close(C, Cref, S, case["key"])
    assert_sums_close(C, g[case["key"] + "_C"], S, case["key"] + " vs reference")


# ------------------------------------------------------------------------------ off-grid operands
@pytest.mark.parametrize("s2n", [True, False])
def test_off_grid_operands_take_exact_path(s2n):
    rng = np.random.default_rng(3)
    A = (rng.standard_normal((96, 40)) * 0.7).astype(np.float32)   # NOT on the FP8 grid
    B = (rng.standard_normal((40, 72)) * 0.05).astype(np.float32)
    tab = g2_table("E4M3", "nocomp")
    fl = orc.flags_of(approx=True, s2n=s2n, qbma=True)
    C = fa().approx_matmul(t(A), t(B), 4, 3, 12, 18, 14, torch.as_tensor(tab), flags=fl).cpu().numpy()
    Cref, S = orc.matmul(A, B, 4, 3, 12, 18, 14, tab, fl, with_abs=True)
    assert_sums_close(C, Cref, S)
    ref = orc.terms(A[:, :4], B[:4], 4, 3, 12, 18, 14, tab, fl)
    for k in range(4):
        Ck = fa().approx_matmul(t(A[:, k:k + 1]), t(B[k:k + 1]), 4, 3, 12, 18, 14, torch.as_tensor(tab), flags=fl)
        assert_terms_equal(Ck.cpu().numpy(), ref[:, k, :], f"k={k}")


# ------------------------------------------------------------------------------ larger / ragged sizes
def _grid_operands(rng, E, M, rows, cols, bias, zero_frac=0.0, scale_bins=8):
    """Random values of the (E, M, bias) grid: codes (expo, mant) drawn with expo in the top
    `scale_bins` codes (subnormals, expo 0, included when E is small), random signs."""
    emax = 2 ** E - 1
    expo = rng.integers(max(0, emax - scale_bins), emax + 1, size=(rows, cols))
    mant = rng.integers(0, 2 ** M, size=(rows, cols))
    v = np.where(expo == 0, np.ldexp(mant / 2 ** M, 1 - bias), np.ldexp(1.0 + mant / 2 ** M, expo - bias))
    v = v * rng.choice([-1.0, 1.0], size=(rows, cols))
    v[rng.random((rows, cols)) < zero_frac] = 0.0
    return v.astype(np.float32)


@pytest.mark.parametrize("shape", [(1, 1, 1), (3, 5, 7), (65, 17, 63), (130, 300, 129), (257, 33, 1000)])
@pytest.mark.parametrize("fmt", [(4, 3, "nocomp"), (3, 4, "comp3"), (2, 5, "nocomp"), (2, 5, "comp3"),
                                 (3, 4, "nocomp")])
def test_ragged_shapes_all_table_modes(shape, fmt):
    E, M, tname = fmt
    Mr, K, N = shape
    rng = np.random.default_rng(Mr * 1000 + K * 10 + N)
    A = _grid_operands(rng, E, M, Mr, K, 2 ** (E - 1) + 2, zero_frac=0.4)
    B = _grid_operands(rng, E, M, K, N, 2 ** (E - 1) + 5)
    bB = rng.integers(2 ** (E - 1) + 4, 2 ** (E - 1) + 7, size=N).astype(np.int32)
    tab = g2_table(f"E{E}M{M}", tname)
    for s2n in (True, False):
        fl = orc.flags_of(approx=True, s2n=s2n, qbma=True)
        C = fa().approx_matmul(t(A), t(B), E, M, 2 ** (E - 1) + 2, t(bB, torch.int32), 2 ** (E - 1) + 4,
                               torch.as_tensor(tab), flags=fl).cpu().numpy()
        Cref, S = orc.matmul(A, B, E, M, 2 ** (E - 1) + 2, bB, 2 ** (E - 1) + 4, tab, fl, with_abs=True)
        assert_sums_close(C, Cref, S, f"{shape} {fmt} s2n={s2n}")


@pytest.mark.parametrize("shape", [(256, 2048, 128), (100, 1000, 70), (64, 4608, 64)])
def test_split_k_matmul(shape):
    """Shapes that fill the GPU in a fraction of a wave take split-K (partials summed in a
    fixed order): sums within tolerance and bit-identical across calls."""
    from fp8_quantization_amd import _lib
    Mr, K, N = shape
    assert _lib.load().fp8a_matmul_workspace_size_mnk(Mr, N, K) > 256, "shape expected to split"
    E, M = 4, 3
    rng = np.random.default_rng(Mr + K + N)
    A = _grid_operands(rng, E, M, Mr, K, 10, zero_frac=0.4)
    B = _grid_operands(rng, E, M, K, N, 13)
    bB = rng.integers(12, 15, size=N).astype(np.int32)
    tab = g2_table("E4M3", "nocomp")
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    run = lambda: fa().approx_matmul(t(A), t(B), E, M, 10, t(bB, torch.int32), 12, torch.as_tensor(tab),
                                     flags=fl).cpu().numpy()
    C1, C2 = run(), run()
    assert np.array_equal(C1.view(np.uint32), C2.view(np.uint32)), "split-K result not deterministic"
    Cref, S = orc.matmul(A, B, E, M, 10, bB, 12, tab, fl, with_abs=True)
    assert_sums_close(C1, Cref, S, f"split-K {shape}")


def test_empty_inner_dimension_gives_zeros():
    A = torch.zeros((5, 0), device=DEV)
    B = torch.zeros((0, 3), device=DEV)
    C = fa().approx_matmul(A, B, 4, 3, 7, 7, 7, None, with_approx=True, with_s2nn2s_opt=True)
    assert C.shape == (5, 3) and torch.count_nonzero(C).item() == 0


# ------------------------------------------------------------------------------ conv
def _im2col_np(x, kh, kw, stride, pad, dil):
    xt = torch.from_numpy(x)
    cols = torch.nn.functional.unfold(xt, (kh, kw), dilation=dil, padding=pad, stride=stride)  # [B, K, L]
    return cols.transpose(1, 2).reshape(-1, cols.shape[1]).numpy()


@pytest.mark.parametrize("cfg", [
    dict(cin=3, cout=64, k=7, s=2, p=3, g=1, hw=32),     # ResNet conv1 shape class, K=147 (ragged)
    dict(cin=16, cout=32, k=3, s=1, p=1, g=1, hw=14),
    dict(cin=16, cout=24, k=1, s=2, p=0, g=1, hw=15),
    dict(cin=8, cout=16, k=3, s=1, p=1, g=4, hw=9),      # grouped, 4 out channels per group
    dict(cin=128, cout=64, k=3, s=1, p=1, g=1, hw=7),    # split-K, hw=49 (scalar reduce)
    dict(cin=256, cout=64, k=3, s=1, p=1, g=2, hw=8),    # split-K, grouped, hw=64 (float4 reduce)
])
def test_conv2d_int_bias_groups(cfg):
    rng = np.random.default_rng(cfg["cin"] * 7 + cfg["cout"])
    E, M = 4, 3
    bA, bR = 9, 12
    x = _grid_operands(rng, E, M, 2 * cfg["cin"], cfg["hw"] * cfg["hw"], bA, zero_frac=0.5)
    x = x.reshape(2, cfg["cin"], cfg["hw"], cfg["hw"])
    cig = cfg["cin"] // cfg["g"]
    w = _grid_operands(rng, E, M, cfg["cout"], cig * cfg["k"] ** 2, 17).reshape(cfg["cout"], cig, cfg["k"], cfg["k"])
    bW = rng.integers(16, 19, size=cfg["cout"]).astype(np.int32)
    tab = g2_table("E4M3", "nocomp")
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    y = fa().approx_conv2d(t(x), t(w), E, M, bA, t(bW, torch.int32), bR, torch.as_tensor(tab), flags=fl,
                           stride=(cfg["s"],) * 2, padding=(cfg["p"],) * 2, groups=cfg["g"]).cpu().numpy()
    cols = _im2col_np(x, cfg["k"], cfg["k"], cfg["s"], cfg["p"], 1)
    Ho = y.shape[2]
    cog = cfg["cout"] // cfg["g"]
    Kg = cig * cfg["k"] ** 2
    for gi in range(cfg["g"]):
        Wg = w[gi * cog:(gi + 1) * cog].reshape(cog, -1).T
        Cref, S = orc.matmul(cols[:, gi * Kg:(gi + 1) * Kg], Wg, E, M, bA, bW[gi * cog:(gi + 1) * cog], bR, tab, fl,
                             with_abs=True)
        got = y[:, gi * cog:(gi + 1) * cog].transpose(0, 2, 3, 1).reshape(-1, cog)
        assert_sums_close(got, Cref, S, f"group {gi}")
    assert y.shape == (2, cfg["cout"], Ho, Ho)


def test_depthwise_conv_tensor_bias_semantics():
    rng = np.random.default_rng(5)
    E, M = 3, 4
    x = _grid_operands(rng, E, M, 2 * 8, 36, 5, zero_frac=0.5).reshape(2, 8, 6, 6)
    w = _grid_operands(rng, E, M, 8, 9, 7).reshape(8, 1, 3, 3)
    bW = np.full(8, 7, np.int32)
    tab = g2_table("E3M4", "comp3")
    for s2n in (False, True):
        fl = orc.flags_of(approx=True, s2n=s2n, qbma=True)
        y = fa().approx_conv2d(t(x), t(w), E, M, torch.tensor([5], device=DEV), t(bW, torch.int32),
                               torch.tensor([6], device=DEV), torch.as_tensor(tab), flags=fl, stride=(1, 1),
                               padding=(1, 1), groups=8).cpu().numpy()
        cols = _im2col_np(x, 3, 3, 1, 1, 1)
        for c in range(8):
            Cref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, 5, 7, 6, tab,
                                 fl | orc.TB, with_abs=True)
            got = y[:, c].reshape(-1, 1)
            assert_sums_close(got, Cref, S, f"channel {c} s2n={s2n}")


@pytest.mark.parametrize("fmt", [(4, 3, "nocomp"), (3, 4, "comp3"), (2, 5, "comp3"), (3, 4, "nocomp")])
@pytest.mark.parametrize("qbma", [True, False])
def test_depthwise_fast_tensor_bias_per_term_bitexact(fmt, qbma):
    """1x1 depthwise: every output is ONE tensor-bias term, so the fast depthwise kernel is
    checked term by term against the oracle, including the expo-0 binade of Q_R and the F7
    band (products near 2^-bR), zeros and every table mode."""
    E, M, tname = fmt
    rng = np.random.default_rng(E * 10 + M + int(qbma))
    bA, bW_, bR = 2 ** (E - 1) + 3, 2 ** (E - 1) + 6, 2 ** (E - 1) + 4
    C = 64
    x = _grid_operands(rng, E, M, 4 * C, 50, bA, zero_frac=0.2, scale_bins=12).reshape(4, C, 5, 10)
    w = _grid_operands(rng, E, M, C, 1, bW_, scale_bins=12).reshape(C, 1, 1, 1)
    # steer some products into the binade [2^-bR, 2^(1-bR)) and onto the F7 band
    w[:8, 0, 0, 0] = np.float32(2.0 ** -bR) / np.where(x[0, :8, 0, 0] == 0, 1, x[0, :8, 0, 0])
    w = np.where(np.isfinite(w), w, 0).astype(np.float32)
    bW = np.full(C, bW_, np.int32)
    tab = g2_table(f"E{E}M{M}", tname)
    fl = orc.flags_of(approx=True, s2n=True, qbma=qbma)
    y = fa().approx_conv2d(t(x), t(w), E, M, torch.tensor([bA], device=DEV), t(bW, torch.int32),
                           torch.tensor([bR], device=DEV), torch.as_tensor(tab), flags=fl, groups=C).cpu().numpy()
    for c in range(C):
        ref = orc.terms(x[:, c].reshape(-1, 1), w[c].reshape(1, 1), E, M, bA, bW[c:c + 1], bR, tab, fl | orc.TB)
        assert_terms_equal(y[:, c].reshape(-1), ref.reshape(-1), f"channel {c}")


def test_depthwise_fast_falls_back_on_off_grid_inputs():
    rng = np.random.default_rng(11)
    E, M = 4, 3
    x = _grid_operands(rng, E, M, 2 * 16, 49, 9, zero_frac=0.3).reshape(2, 16, 7, 7)
    x[1, 3, 2, 2] = 0.123456  # not an E4M3 value
    w = _grid_operands(rng, E, M, 16, 9, 12).reshape(16, 1, 3, 3)
    bW = np.full(16, 12, np.int32)
    tab = g2_table("E4M3", "nocomp")
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    y = fa().approx_conv2d(t(x), t(w), E, M, torch.tensor([9], device=DEV), t(bW, torch.int32),
                           torch.tensor([10], device=DEV), torch.as_tensor(tab), flags=fl, padding=(1, 1),
                           groups=16).cpu().numpy()
    cols = _im2col_np(x, 3, 3, 1, 1, 1)
    for c in range(16):
        Cref, S = orc.matmul(cols[:, c * 9:(c + 1) * 9], w[c].reshape(9, 1), E, M, 9, 12, 10, tab, fl | orc.TB,
                             with_abs=True)
        assert_sums_close(y[:, c].reshape(-1, 1), Cref, S, f"channel {c}")


# ------------------------------------------------------------------------------ FP8 fake quant
@pytest.mark.parametrize("M", [3, 4, 5, 2])
def test_fp8_fake_quantize_matches_oracle(M):
    rng = np.random.default_rng(M)
    x = (rng.standard_normal((6, 500)) * np.exp(rng.standard_normal((6, 1)))).astype(np.float32)
    mx = np.abs(x).max(axis=1).astype(np.float32)
    y, b = fa().fp8_fake_quantize(t(x), t(mx), 8, M, per_row=True)
    yr, br = orc.fp8_fake_quant(x, mx, 7 - M, M, per_row=True)
    np.testing.assert_array_equal(b.cpu().numpy().reshape(-1), br)
    np.testing.assert_array_equal(y.cpu().numpy().view(np.uint32), yr.view(np.uint32))
    y1, b1 = fa().fp8_fake_quantize(t(x), t(mx[:1]), 8, M, per_row=False)
    yr1, br1 = orc.fp8_fake_quant(x, mx[:1], 7 - M, M, per_row=False)
    np.testing.assert_array_equal(y1.cpu().numpy().view(np.uint32), yr1.view(np.uint32))


@pytest.mark.parametrize("scale", [1e-38, 1e-33, 1e-25, 1e25, 1e33])
def test_fp8_fake_quantize_extreme_ranges(scale):
    """Ranges where the quantization step 2^k leaves the reciprocal's range (k < -126: the
    kernel divides) or sits next to it (it multiplies by 2^-k): same bits as the oracle."""
    rng = np.random.default_rng(int(np.log10(scale)) + 60)
    x = (rng.standard_normal((4, 300)) * scale).astype(np.float32)
    x[:, :5] = [0.0, -0.0, scale, -scale, scale * 1e-3]
    mx = (np.abs(x).max(axis=1) * np.array([1.0, 0.5, 2.0, 1e-3])).astype(np.float32)
    for M in (3, 4):
        y, b = fa().fp8_fake_quantize(t(x), t(mx), 8, M, per_row=True)
        yr, br = orc.fp8_fake_quant(x, mx, 7 - M, M, per_row=True)
        np.testing.assert_array_equal(b.cpu().numpy().reshape(-1), br)
        np.testing.assert_array_equal(y.cpu().numpy().view(np.uint32), yr.view(np.uint32))


@pytest.mark.parametrize("M", [2, 3, 4, 5])
@pytest.mark.parametrize("mxv", [6.0, 0.37, 448.0, 3e-3])
def test_fp8_fake_quantize_ties_and_binade_edges(M, mxv):
    """Exact ties (the midpoint between two grid values) and values next to them, in every binade of
    the quantizer from below its smallest normal one up to maxval, zero and float subnormals, both
    signs: the kernel's bit-level rounding (fq_apply) against the oracle's literal formula."""
    E = 7 - M
    bias = float(np.rint(2 ** E - np.log2(mxv) + np.log2(2 - 2.0 ** -M) - 1))
    vals = [0.0, -0.0, 1e-45, -1e-45, 1e-40, 1.17549435e-38, mxv, -mxv, mxv * 1.5, np.nextafter(np.float32(mxv), 0)]
    for ls in range(1, int(2 ** E + 2)):
        q = 2.0 ** (max(ls, 1) - M - bias)
        for m in range(2 ** M, 2 ** (M + 1), max(1, 2 ** M // 8)):
            for tie in (m + 0.5, m + 1.5):
                v = np.float32(tie * q)
                vals += [v, np.nextafter(v, np.float32(np.inf)), np.nextafter(v, np.float32(0)), -v]
        for m in range(0, 2 ** M):  # the fixed-quantum band below the smallest normal binade
            v = np.float32((m + 0.5) * 2.0 ** (1 - M - bias))
            vals += [v, -v, np.nextafter(v, np.float32(np.inf))]
    x = np.array(vals, dtype=np.float32).reshape(1, -1)
    mx = np.array([mxv], np.float32)
    y, b = fa().fp8_fake_quantize(t(x), t(mx), 8, M, per_row=False)
    yr, br = orc.fp8_fake_quant(x, mx, E, M, per_row=False)
    np.testing.assert_array_equal(b.cpu().numpy().reshape(-1), br)
    np.testing.assert_array_equal(y.cpu().numpy().view(np.uint32), yr.view(np.uint32))


# ------------------------------------------------------------------------------ qamaa
@pytest.mark.parametrize("case", META["g6"], ids=lambda c: c["key"])
def test_qamaa_matmul(case):
    """Bit-exact vs the oracle (same float32 k-order sums); vs the reference identical up to
    one FP8 step where its torch-order sum straddles a rounding boundary (none in G6)."""
    g = gio.load("g6_qamaa.npz")
    A, B = g[case["fmt"] + "_A"], g[case["fmt"] + "_B"]
    mx = torch.tensor([case["maxval"]], device=DEV)
    C = fa().qamaa_matmul(t(A), t(B), mx, 8, case["M"]).cpu().numpy()
    Cref, _ = orc.matmul_qamaa(A, B, case["maxval"], 8, case["M"])
    np.testing.assert_array_equal(C, Cref)
    np.testing.assert_array_equal(C, g[case["key"] + "_C"])


@pytest.mark.parametrize("groups", [1, 2])
def test_qamaa_conv2d(groups):
    rng = np.random.default_rng(11 + groups)
    x = _grid_operands(rng, 3, 4, 2 * 8, 100, 6, zero_frac=0.4).reshape(2, 8, 10, 10)
    w = _grid_operands(rng, 3, 4, 12, (8 // groups) * 9, 8).reshape(12, 8 // groups, 3, 3)
    y = fa().qamaa_conv2d(t(x), t(w), torch.tensor([2.5], device=DEV), 8, 4, stride=(1, 1), padding=(1, 1),
                          groups=groups).cpu().numpy()
    cols = _im2col_np(x, 3, 3, 1, 1, 1)
    cog, Kg = 12 // groups, (8 // groups) * 9
    for gi in range(groups):
        Cref, _ = orc.matmul_qamaa(cols[:, gi * Kg:(gi + 1) * Kg], w[gi * cog:(gi + 1) * cog].reshape(cog, -1).T, 2.5,
                                   8, 4)
        got = y[:, gi * cog:(gi + 1) * cog].transpose(0, 2, 3, 1).reshape(-1, cog)
        np.testing.assert_array_equal(got, Cref)
