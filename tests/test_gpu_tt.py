"""The tile-table kernel for E3M4 / E2M5 (gemm_tt_kernel, csrc/gemm_tt.h).

Every case reads the launch's flag word back and asserts it is 0, i.e. the pre-decoded
tile-table path produced the result (not the gated exact kernel).  Covered, for both formats and
every error table the reference selects for them (withComp False: E3M4 entries 0..3, E2M5 0..5;
withComp True, dnsmp 3: entries -1..1, which make the F7 sign rule observable -- E3M4 runs its
F7 form, E2M5 with a signed table stays on gemm_fast_kernel and is checked here all the same)
and no table:
  * every code pair of the format (both signs, subnormals, zeros) as a single-term product, bit-exact
    against the oracle's terms, at bias triples that put the result grid's floor inside the
    products' range (flush, subnormal band and normal results all occur);
  * implicit-GEMM convs with padding (the zero-bordered word image), stride, dilation, groups,
    ragged M / N and split-K against the oracle on unfolded inputs, run-to-run bit-identity;
  * the matrix form with lda > K and a column-strided B;
  * an off-grid activation raises the flag and the exact kernel's result is returned.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio
from fp8_quantization_amd.error_tables import get_error_table_NN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FMTS = [(3, 4), (2, 5)]


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _table(E, M, kind):
    if kind == "none":
        return np.zeros((1 << M, 1 << M), np.int32)
    return get_error_table_NN(E, M, withComp=(kind == "comp"), dnsmp_factor=3).numpy().astype(np.int32)


def _flags(kind):
    return orc.flags_of(approx=kind != "none", s2n=True, qbma=True)


def _all_codes(E, M, bias):
    """Every value of the (E, M) format at the given bias, both signs (zeros included)."""
    e = np.repeat(np.arange(1 << E), 1 << M)
    m = np.tile(np.arange(1 << M), 1 << E)
    v = np.where(e == 0, np.ldexp(m / 2.0 ** M, 1 - bias), np.ldexp(1.0 + m / 2.0 ** M, e - bias))
    return np.concatenate([v, -v]).astype(np.float32)


def _grid(rng, E, M, shape, bias, zero_frac=0.0, sub_frac=0.05):
    emax = (1 << E) - 1
    bias = np.broadcast_to(np.asarray(bias), shape)
    expo = rng.integers(1, emax + 1, size=shape)
    mant = rng.integers(0, 1 << M, size=shape)
    v = np.ldexp(1.0 + mant / 2.0 ** M, expo - bias)
    sub = rng.random(shape) < sub_frac
    v[sub] = np.ldexp(rng.integers(1, 1 << M, size=shape) / 2.0 ** M, 1 - bias)[sub]
    v = v * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype=dtype, device=DEV)


def _matmul_raw(A, lda, B, sbk, sbn, Mr, N, K, E, M, bA, bB, bR, table, flags):
    from fp8_quantization_amd import _lib
    L = _lib.load()
    At, Bt = _dev(A), _dev(B)
    C = torch.empty((Mr, N), dtype=torch.float32, device=DEV)
    ws = torch.zeros(int(L.fp8a_matmul_workspace_size_mnk(Mr, N, K)), dtype=torch.uint8, device=DEV)
    bB = np.array(np.broadcast_to(np.asarray(bB, np.int32), (N,)))
    tA, tB, tR = _dev([bA], torch.int32), _dev(bB, torch.int32), _dev([bR], torch.int32)
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32))
    rc = L.fp8a_matmul(_lib.dev_ptr(At), lda, _lib.dev_ptr(Bt), sbk, sbn, _lib.dev_ptr(C), N, Mr, N, K, E, M,
                       _lib.dev_ptr(tA), _lib.dev_ptr(tB), 1, _lib.dev_ptr(tR), _lib.host_ptr(tab), flags,
                       _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_matmul")
    torch.cuda.synchronize()
    return C.cpu().numpy(), int(ws[:4].view(torch.int32).item())


def _conv_raw(x, w, E, M, bA, bW, bR, table, flags, stride, pad, dil, groups):
    from fp8_quantization_amd import _lib
    L = _lib.load()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * pad - dil * (kh - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (kw - 1) - 1) // stride + 1
    xt, wt = _dev(x), _dev(w)
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=DEV)
    need = int(L.fp8a_conv2d_workspace_size(Bn, Cin, H, W, Cout, kh, kw, stride, stride, pad, pad, dil, dil, groups))
    ws = torch.zeros(need, dtype=torch.uint8, device=DEV)
    tA, tW, tR = _dev([bA], torch.int32), _dev(bW, torch.int32), _dev([bR], torch.int32)
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32))
    rc = L.fp8a_conv2d(_lib.dev_ptr(xt), _lib.dev_ptr(wt), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw, stride,
                       stride, pad, pad, dil, dil, groups, E, M, _lib.dev_ptr(tA), _lib.dev_ptr(tW), _lib.dev_ptr(tR),
                       _lib.host_ptr(tab), flags, _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_conv2d")
    torch.cuda.synchronize()
    return y.cpu().numpy(), int(ws[:4].view(torch.int32).item())


def _conv_ref(x, w, E, M, bA, bW, bR, table, flags, stride, pad, dil, groups):
    Cout, cig, kh, kw = w.shape
    cols = torch.nn.functional.unfold(torch.from_numpy(x), (kh, kw), dilation=dil, padding=pad, stride=stride)
    cols = cols.transpose(1, 2).reshape(-1, cols.shape[1]).numpy()
    cog, Kg = Cout // groups, cig * kh * kw
    outs, sums = [], []
    for g in range(groups):
        Wg = w[g * cog:(g + 1) * cog].reshape(cog, -1).T
        C, S = orc.matmul(cols[:, g * Kg:(g + 1) * Kg], Wg, E, M, bA, bW[g * cog:(g + 1) * cog], bR, table, flags,
                          with_abs=True)
        outs.append(C)
        sums.append(S)
    return np.concatenate(outs, 1), np.concatenate(sums, 1)


def _close(got, ref, S, what=""):
    bad = np.abs(got.astype(np.float64) - ref) > gio.sum_tolerance(S.astype(np.float64))
    assert not bad.any(), f"{what}: {np.count_nonzero(bad)} outputs outside the bar"


def _terms_equal(got, ref):
    same = (got.view(np.uint32) == ref.view(np.uint32)) | ((got == 0) & (ref == 0))
    if not same.all():
        i = tuple(np.argwhere(~same)[0])
        raise AssertionError(f"{np.count_nonzero(~same)} terms differ; first at {i}: got {got[i]!r} ref {ref[i]!r}")


@pytest.mark.parametrize("kind", ["nocomp", "comp", "none"])
@pytest.mark.parametrize("fmt", FMTS, ids=["E3M4", "E2M5"])
@pytest.mark.parametrize("shift", [0, 3, 6])
def test_every_code_pair_bitexact(fmt, kind, shift):
    """All (2 x 2^(E+M))^2 code pairs as K = 1 products.  bR = bA + bB - shift - base puts the
    result grid's floor among the products: flushes, the subnormal band (incl. the F7 interval
    for the signed tables) and normal results all occur."""
    E, M = fmt
    bA, bB = (1 << (E - 1)) + 2, (1 << (E - 1)) + 5
    bR = bA + bB - (1 << E) - shift
    # K = 256 with one nonzero K-step: each output is exactly one term, and K is long enough for
    # E3M4's packed-f16 form (run_gemm picks it for K >= 64 -- option tt16_mink -- or a signed table)
    a = _all_codes(E, M, bA).reshape(-1, 1)
    b = _all_codes(E, M, bB).reshape(1, -1)
    K = 256
    A = np.zeros((a.shape[0], K), np.float32)
    A[:, 0] = a[:, 0]
    B = np.zeros((K, b.shape[1]), np.float32)
    B[0] = b[0]
    tab, fl = _table(E, M, kind), _flags(kind)
    C, flag = _matmul_raw(A, K, B, B.shape[1], 1, A.shape[0], B.shape[1], K, E, M, bA, bB, bR, tab, fl)
    assert flag == 0, "fallback flag raised: the tile-table path did not produce these terms"
    ref = orc.terms(a, b, E, M, bA, bB, bR, tab, fl)[:, 0, :]
    _terms_equal(C, ref)


CONVS = [
    dict(B=2, cin=3, cout=64, k=7, s=2, p=3, d=1, g=1, hw=30),     # conv1 class, padding 3
    dict(B=3, cin=16, cout=40, k=3, s=1, p=1, d=1, g=1, hw=13),    # ragged M (507), N (40), padding 1
    dict(B=2, cin=24, cout=72, k=3, s=2, p=2, d=2, g=1, hw=17),    # dilation, N > 64
    dict(B=2, cin=32, cout=48, k=1, s=2, p=0, d=1, g=1, hw=15),    # 1x1 downsample class, no padding
    dict(B=2, cin=16, cout=32, k=3, s=1, p=1, d=1, g=2, hw=9),     # groups
    dict(B=1, cin=256, cout=128, k=3, s=1, p=1, d=1, g=1, hw=7),   # split-K (K = 2304)
]


@pytest.mark.parametrize("kind", ["nocomp", "comp"])
@pytest.mark.parametrize("fmt", FMTS, ids=["E3M4", "E2M5"])
@pytest.mark.parametrize("cfg", CONVS, ids=[f"c{i}" for i in range(len(CONVS))])
def test_conv_matches_oracle(cfg, fmt, kind):
    E, M = fmt
    rng = np.random.default_rng(cfg["cin"] * 31 + cfg["cout"] + E)
    bA, bR = (1 << (E - 1)) + 3, (1 << (E - 1)) + 4
    x = _grid(rng, E, M, (cfg["B"], cfg["cin"], cfg["hw"], cfg["hw"]), bA, zero_frac=0.45)
    cig = cfg["cin"] // cfg["g"]
    bW = rng.integers((1 << (E - 1)) + 5, (1 << (E - 1)) + 8, size=cfg["cout"]).astype(np.int32)
    w = _grid(rng, E, M, (cfg["cout"], cig, cfg["k"], cfg["k"]), bW[:, None, None, None])
    args = (cfg["s"], cfg["p"], cfg["d"], cfg["g"])
    tab, fl = _table(E, M, kind), _flags(kind)
    y, flag = _conv_raw(x, w, E, M, bA, bW, bR, tab, fl, *args)
    assert flag == 0, "fallback flag raised: the tile-table path did not produce this result"
    ref, S = _conv_ref(x, w, E, M, bA, bW, bR, tab, fl, *args)
    _close(y.transpose(0, 2, 3, 1).reshape(-1, y.shape[1]), ref, S, str(cfg))
    y2, _ = _conv_raw(x, w, E, M, bA, bW, bR, tab, fl, *args)
    assert np.array_equal(y.view(np.uint32), y2.view(np.uint32)), "not deterministic"


@pytest.mark.parametrize("fmt", FMTS, ids=["E3M4", "E2M5"])
@pytest.mark.parametrize("shape", [(130, 300, 129), (64, 4608, 64), (257, 17, 5)])
def test_matmul_strided_operands(shape, fmt):
    E, M = fmt
    Mr, K, N = shape
    rng = np.random.default_rng(Mr + K + N + E)
    bA, bR = (1 << (E - 1)) + 3, (1 << (E - 1)) + 4
    lda = K + 7
    Afull = _grid(rng, E, M, (Mr, lda), bA, zero_frac=0.4)
    bB = rng.integers((1 << (E - 1)) + 5, (1 << (E - 1)) + 8, size=N).astype(np.int32)
    W = _grid(rng, E, M, (N, K), bB[:, None])
    tab, fl = _table(E, M, "comp"), _flags("comp")
    C, flag = _matmul_raw(Afull, lda, W, 1, K, Mr, N, K, E, M, bA, bB, bR, tab, fl)
    assert flag == 0
    ref, S = orc.matmul(Afull[:, :K], W.T, E, M, bA, bB, bR, tab, fl, with_abs=True)
    _close(C, ref, S, str(shape))


@pytest.mark.parametrize("fmt", FMTS, ids=["E3M4", "E2M5"])
def test_off_grid_operand_falls_back(fmt):
    E, M = fmt
    rng = np.random.default_rng(3)
    bA, bR = (1 << (E - 1)) + 3, (1 << (E - 1)) + 4
    x = _grid(rng, E, M, (2, 16, 9, 9), bA, zero_frac=0.3)
    bW = np.full(32, (1 << (E - 1)) + 6, np.int32)
    w = _grid(rng, E, M, (32, 16, 3, 3), bW[0])
    x[1, 3, 4, 4] = 0.3001  # off the (M, bA) grid
    tab, fl = _table(E, M, "nocomp"), _flags("nocomp")
    y, flag = _conv_raw(x, w, E, M, bA, bW, bR, tab, fl, 1, 1, 1, 1)
    assert flag != 0, "pre-decode did not flag the launch"
    ref, S = _conv_ref(x, w, E, M, bA, bW, bR, tab, fl, 1, 1, 1, 1)
    _close(y.transpose(0, 2, 3, 1).reshape(-1, y.shape[1]), ref, S, "off-grid")


# E3M4 runs the packed-f16 form (gemm_tt16_kernel): per 64-column tile the frame
# shift S = min(min bB - 7, bR - bA + 9) must give Emn = bA - bR + S >= -10 and
# max bB <= S + 13; a tile outside that window sets a flag bit (2: Emn, 16: the bB spread) and
# the f32 form (gemm_tt_kernel on the same pre-decoded operands) reruns the launch.  bB offsets
# are relative to min bB.
WINDOW = [
    ("edge_bR_high", [0] * 64, 3, 0),             # bR = bA + bB + 3: Emn = -10, inside
    ("bR_too_high", [0] * 64, 4, 2),              # bR = bA + bB + 4: Emn = -11
    ("bR_low", [0] * 64, -17, 0),                 # the S = bR - bA + 9 branch (Emn = 9)
    ("spread_6", [0] * 32 + [6] * 32, 0, 0),      # max bB = S + 13
    ("spread_7", [0] * 32 + [7] * 32, 0, 16),     # a column's smallest c_b' falls below 2^-16
]


@pytest.mark.parametrize("kind", ["nocomp", "comp"])
@pytest.mark.parametrize("case", WINDOW, ids=[w[0] for w in WINDOW])
def test_e3m4_f16_window(case, kind):
    name, boffs, rdelta, want_flag = case
    E, M = 3, 4
    rng = np.random.default_rng(len(name) * 7 + (kind == "comp"))
    bA = 7
    bB = np.array([bA + o for o in boffs], np.int32)
    bR = int(bA + bB.min() + rdelta)
    Mr, K, N = 96, 256, 64  # K >= 64: the packed-f16 form for both table kinds
    A = _grid(rng, E, M, (Mr, K), bA, zero_frac=0.2, sub_frac=0.1)
    W = _grid(rng, E, M, (N, K), bB[:, None], zero_frac=0.1, sub_frac=0.1)
    tab, fl = _table(E, M, kind), _flags(kind)
    C, flag = _matmul_raw(A, K, W, 1, K, Mr, N, K, E, M, bA, bB, bR, tab, fl)
    assert flag == want_flag, f"{name}: flag {flag}"
    ref, S = orc.matmul(A, W.T, E, M, bA, bB, bR, tab, fl, with_abs=True)
    _close(C, ref, S, name)


@pytest.mark.parametrize("kind", ["nocomp", "comp"])
def test_e3m4_above_top_binade_takes_f32_form(kind):
    """An activation two binades above the format's largest one (the quantizer's rint bias allows
    one: 5.0 at bA = 6 is inside) is on the mantissa grid but outside the f16 window: flag bit 2,
    and the f32 form's result (which matches the oracle) is returned."""
    E, M = 3, 4
    rng = np.random.default_rng(11)
    bA, bR = 6, 4
    bB = np.full(64, 10, np.int32)
    K = 256
    A = _grid(rng, E, M, (80, K), bA, zero_frac=0.2)
    A[3, 5] = 10.0
    A[70, 40] = -13.0
    A[71, 41] = 5.0
    W = _grid(rng, E, M, (64, K), bB[:, None], zero_frac=0.1)
    tab, fl = _table(E, M, kind), _flags(kind)
    C, flag = _matmul_raw(A, K, W, 1, K, 80, 64, K, E, M, bA, bB, bR, tab, fl)
    assert flag == 4, f"flag {flag}"
    ref, S = orc.matmul(A, W.T, E, M, bA, bB, bR, tab, fl, with_abs=True)
    _close(C, ref, S, "above top binade")


@pytest.mark.parametrize("regime", ["band", "zero", "mixed"])
@pytest.mark.parametrize("fmt,kind", [((2, 5), "nocomp"), ((2, 5), "none"), ((3, 4), "nocomp")],
                         ids=["E2M5", "E2M5-notable", "E3M4"])
def test_band_and_zero_wave_tiles_bit_identical(fmt, kind, regime):
    """gemm_tt_kernel's band / zero wave-tile forms (round 6, csrc/gemm_tt.h): a staged tile whose
    products all lie below the result grid's smallest normal takes fma(t, c_a, cmin) - cmin per
    term, one whose products all lie below half the subnormal quantum adds nothing.  Results are
    bit-identical to the general form (option tt_band 0), within the sum bar of the oracle, and the
    terms are bit-exact (a K-step-sparse layout makes every output one term).  E3M4 at K = 48 runs
    gemm_tt_kernel<4> (the packed-f16 form starts at K = 64)."""
    from fp8_quantization_amd import _lib
    E, M = fmt
    import zlib
    rng = np.random.default_rng(zlib.crc32(f"{E}{kind}{regime}".encode()))
    bA = (1 << (E - 1)) + 2
    Mr, K, N = 300, 48 if E == 3 else 160, 80
    A = _grid(rng, E, M, (Mr, K), bA, zero_frac=0.4)
    bB = rng.integers((1 << (E - 1)) + 5, (1 << (E - 1)) + 8, size=N).astype(np.int32)
    W = _grid(rng, E, M, (N, K), bB[:, None])
    top = (1 << E) - bA + int((1 << E) - bB.min())  # >= the largest e_a + e_b + 2: |a b| < 2^top
    # band: 2^top <= the grid's smallest normal 2^(1 - bR); zero: 2^top <= half its quantum 2^(-bR - M)
    bR = {"band": 1 - top, "zero": -top - M, "mixed": bA + 2}[regime]
    tab, fl = _table(E, M, kind), _flags(kind)
    old = _lib.set_option("tt_band", 1)
    try:
        C1, f1 = _matmul_raw(A, K, W, 1, K, Mr, N, K, E, M, bA, bB, bR, tab, fl)
        _lib.set_option("tt_band", 0)
        C0, f0 = _matmul_raw(A, K, W, 1, K, Mr, N, K, E, M, bA, bB, bR, tab, fl)
    finally:
        _lib.set_option("tt_band", old)
    assert f1 == 0 and f0 == 0
    assert np.array_equal(C1.view(np.uint32), C0.view(np.uint32)), "band forms differ from the general form"
    ref, S = orc.matmul(A, W.T, E, M, bA, bB, bR, tab, fl, with_abs=True)
    _close(C1, ref, S, regime)
    if regime == "zero":
        assert not np.any(C1), "every product is below half the quantum: every term is 0"
    # terms: one nonzero K-step per row (the others zero), so each output is a single term
    As = np.zeros_like(A)
    ks = rng.integers(0, K, size=Mr)
    As[np.arange(Mr), ks] = A[np.arange(Mr), ks]
    Ct, ft = _matmul_raw(As, K, W, 1, K, Mr, N, K, E, M, bA, bB, bR, tab, fl)
    assert ft == 0
    T = orc.terms(As, W.T, E, M, bA, bB, bR, tab, fl)  # [Mr, K, N]
    _terms_equal(Ct, T[np.arange(Mr), ks, :])
