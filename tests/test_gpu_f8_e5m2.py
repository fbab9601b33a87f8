"""E5M2 on the matrix-core path (round 4): gemm_f8mx_kernel<.., XF = 1>.

The E5M2 result grid of bias bR is the OCP e5m2 (bf8) grid scaled by 2^(15-bR), so the same
tile-table kernel as E4M3 rounds each term with v_cvt_scalef32_pk_bf8_bf16 and sums the bf8
codes on the matrix core.  The reference has no E5M2 error table and
raises (approx_matmul_whole_v9.py:588-590), so the parity pin is the oracle's restatement of the
v9 term (itself pinned to the reference's E5M2 G1 / G2 fixtures, tests/test_oracle_golden.py).
Checked here:
  * every one of the 256 x 256 E5M2 code pairs as a K = 1 product, bit-exact against the oracle,
    for bias triples spanning the subnormal band, the flush-to-zero region and the grid's top
    binade, with the launch's path (f8mx) and its fallback flag read back;
  * terms beyond the e5m2 range raise the flag and the exact kernel's terms are returned;
  * sums at conv-like shapes (split-K, ragged tiles, narrow N) within the 1e-5 * sum|term| bar.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
E, M = 5, 2


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


def _all_codes(bias):
    """The 256 E5M2 values of the given bias (both zeros included)."""
    e = np.repeat(np.arange(32), 4)
    m = np.tile(np.arange(4), 32)
    v = np.where(e == 0, np.ldexp(m / 4.0, 1 - bias), np.ldexp(1.0 + m / 4.0, e - bias))
    return np.concatenate([v, -v]).astype(np.float32)


FB_ANY, FB_HALF = 1, 64  # the flag word's exact-fallback / halved-block bits (csrc/fp8approx.hip)


def _matmul_raw(A, B, bA, bB, bR, table, flags):
    """fp8a_matmul (E5M2) through ctypes with a caller-owned workspace: (C, flag word, paths)."""
    from fp8_quantization_amd import _lib
    L = _lib.load()
    A = torch.from_numpy(np.ascontiguousarray(A)).to(DEV)
    B = torch.from_numpy(np.ascontiguousarray(B)).to(DEV)
    Mr, K = A.shape
    N = B.shape[1]
    C = torch.empty((Mr, N), dtype=torch.float32, device=DEV)
    ws = torch.zeros(max(int(L.fp8a_matmul_workspace_size_mnk(Mr, N, K)), 256), dtype=torch.uint8, device=DEV)
    tA = torch.tensor([bA], dtype=torch.int32, device=DEV)
    tB = torch.as_tensor(np.asarray(bB, np.int32).reshape(-1)).to(DEV)
    tR = torch.tensor([bR], dtype=torch.int32, device=DEV)
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32))
    _lib.path_stats(reset=True)
    rc = L.fp8a_matmul(_lib.dev_ptr(A), K, _lib.dev_ptr(B), N, 1, _lib.dev_ptr(C), N, Mr, N, K, E, M,
                       _lib.dev_ptr(tA), _lib.dev_ptr(tB), 0 if tB.numel() == 1 else 1, _lib.dev_ptr(tR),
                       _lib.host_ptr(tab), flags, _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_matmul")
    torch.cuda.synchronize()
    flag = int(ws[:4].view(torch.int32).item())
    return C.cpu().numpy(), flag, _lib.path_stats(reset=True)


def _terms_equal(got, ref):
    same = (got.view(np.uint32) == ref.view(np.uint32)) | ((got == 0) & (ref == 0))
    if not same.all():
        i = tuple(np.argwhere(~same)[0])
        raise AssertionError(f"{np.count_nonzero(~same)} terms differ; first at {i}: got {got[i]!r} ref {ref[i]!r}")


def _table(kind):
    if kind == "zero":
        return gio.load("g2_matmul.npz")["E5M2_table_zero"]
    # a {0,1} table (no reference E5M2 table has one: an extension the kernel supports, pinned by
    # the oracle only)
    return np.array([[0, 1, 0, 1], [1, 0, 1, 0], [0, 0, 1, 1], [1, 1, 0, 0]], np.int32)


# bA + bB - bR >= 33: every product fits the e5m2 range (the grid's normal binades 1-bR .. 30-bR)
@pytest.mark.parametrize("biases", [(20, 20, 7), (18, 22, 5), (24, 24, 15), (16, 17, 0), (10, 10, -13),
                                    (30, 12, 9)])
@pytest.mark.parametrize("table,approx", [("zero", True), ("zero", False), ("w1", True)])
def test_every_code_pair_bitexact(biases, table, approx):
    bA, bB, bR = biases
    A = _all_codes(bA).reshape(-1, 1)
    B = _all_codes(bB).reshape(1, -1)
    tab = _table(table)
    fl = orc.flags_of(approx=approx, s2n=True, qbma=True)
    C, flag, paths = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    _terms_equal(C, orc.terms(A, B, E, M, bA, bB, bR, tab, fl)[:, 0, :])
    assert paths["f8mx"] == 1, paths
    assert flag == 0, "fallback flag raised: the bf8 form did not produce these terms"


def test_terms_beyond_e5m2_range():
    """Products above binade 30 - bR (Q_R lets the exponent run past max_norm, F6) convert to
    inf / NaN: the tile is flagged and the exact kernel's terms come back."""
    bA, bB, bR = 16, 16, 5
    A = _all_codes(bA).reshape(-1, 1)
    B = _all_codes(bB).reshape(1, -1)
    tab = _table("zero")
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    C, flag, paths = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    assert flag != 0 and paths["f8mx"] == 1
    _terms_equal(C, orc.terms(A, B, E, M, bA, bB, bR, tab, fl)[:, 0, :])


def _grid(rng, shape, bias, zero_frac=0.0, top=10):
    expo = rng.integers(31 - top, 32, size=shape)
    mant = rng.integers(0, 4, size=shape)
    v = np.ldexp(1.0 + mant / 4.0, expo - bias) * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


@pytest.mark.parametrize("shape", [(300, 1152, 64), (129, 577, 24), (64, 4608, 16), (1000, 96, 160), (33, 7, 5)])
def test_sums_within_bar(shape):
    Mr, K, N = shape
    rng = np.random.default_rng(Mr + K + N)
    bA, bR = 22, 14
    A = _grid(rng, (Mr, K), bA, zero_frac=0.5)
    B = _grid(rng, (K, N), 26)
    bB = rng.integers(25, 28, size=N).astype(np.int32)
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    tab = _table("zero")
    C, _, paths = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    assert paths["f8mx"] == 1, paths
    ref, S = orc.matmul(A, B, E, M, bA, bB, bR, tab, fl, with_abs=True)
    assert np.all(np.abs(C.astype(np.float64) - ref) <= gio.sum_tolerance(S))


def _codes_from(bias, min_field):
    """The E5M2 values of the given bias whose exponent field is >= min_field (both signs)."""
    e = np.repeat(np.arange(min_field, 32), 4)
    m = np.tile(np.arange(4), 32 - min_field)
    v = np.ldexp(1.0 + m / 4.0, e - bias)
    return np.concatenate([v, -v]).astype(np.float32)


def test_top_binade_terms_without_fallback():
    """The E5M2 result grid's top binade 31 - bR (e5m2's exponent 31 is inf / NaN): an A element
    whose products reach it is converted one binade down and its MX block scaled by 2 -- bit-exact
    terms with NO fallback, as long as its products stay at or above the grid's second binade
    (here: every A code against B codes of exponent field >= 16, bA + bB - bR = 32)."""
    bA, bB, bR = 20, 20, 8
    A = _all_codes(bA).reshape(-1, 1)
    B = _codes_from(bB, 16).reshape(1, -1)
    tab = _table("zero")
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    ref = orc.terms(A, B, E, M, bA, bB, bR, tab, fl)[:, 0, :]
    assert np.abs(ref).max() >= 2.0 ** (31 - bR), "the case must reach the top binade"
    C, flag, paths = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    _terms_equal(C, ref)
    # the plain form's tiles went to the halved-block form (FB_HALF), none to the exact kernel
    assert paths["f8mx"] == 1 and flag & FB_ANY == 0 and flag & FB_HALF, flag


@pytest.mark.parametrize("mixed", [False, True])
def test_top_binade_sums(mixed):
    """Sums with top-binade products: moderate A (halvable everywhere: no fallback) or A mixing
    very large and tiny values in one MX block (those tiles fall back): within the bar either way."""
    rng = np.random.default_rng(11 + mixed)
    bA, bB, bR = 20, 20, 8
    Mr, K, N = 256, 96, 48
    ea = rng.integers(25, 32, size=(Mr, K)) if not mixed else np.where(rng.random((Mr, K)) < 0.5,
                                                                        rng.integers(28, 32, size=(Mr, K)),
                                                                        rng.integers(0, 4, size=(Mr, K)))
    A = np.where(ea == 0, np.ldexp(rng.integers(0, 4, size=(Mr, K)) / 4.0, 1 - bA),
                 np.ldexp(1.0 + rng.integers(0, 4, size=(Mr, K)) / 4.0, ea - bA))
    A = (A * rng.choice([-1.0, 1.0], size=(Mr, K))).astype(np.float32)
    B = (np.ldexp(1.0 + rng.integers(0, 4, size=(K, N)) / 4.0, rng.integers(16, 32, size=(K, N)) - bB)
         * rng.choice([-1.0, 1.0], size=(K, N))).astype(np.float32)
    tab = _table("zero")
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    C, flag, paths = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    assert paths["f8mx"] == 1
    if not mixed:
        assert flag & FB_ANY == 0, flag
    ref, S = orc.matmul(A, B, E, M, bA, bB, bR, tab, fl, with_abs=True)
    assert np.all(np.abs(C.astype(np.float64) - ref) <= gio.sum_tolerance(S))
