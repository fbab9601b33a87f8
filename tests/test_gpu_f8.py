"""The E4M3 LUT + hardware-fp8 form of the fast kernel (TM_F8).

For E4M3 with s2n and per-product quantization and a {0,1} (or no) error table, the term
Q_R(a*b - T*c_a*c_b*2^-M) is computed as a clamped LDS table value V'(sign a, m_a, m_b) times
c_b, rounded by the gfx950 scaled fp8 conversion.  Checked here:
  * every one of the 256 x 256 E4M3 code pairs as a K = 1 product (one term per output),
    bit-exact against the oracle, for several bias triples, with the launch's fallback flag
    read back to prove the fast form (not the exact kernel) produced them;
  * terms beyond the e4m3 range raise the flag and the exact kernel's result is returned;
  * a fallback recomputes only the affected 64 x 64 output units (one out-of-range term: its
    tile; an off-grid A element: its row unit; an off-grid B element: its column unit) and
    every other output is bit-identical to the fast path's, with the library's fallback
    counters (fp8a_fallback_stats) recording the units;
  * sums at realistic shapes stay within the 1e-5 * sum|term| bar.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fp8_quantization_amd import _lib
    _lib.load()


@pytest.fixture
def path():
    """The E4M3 per-pair matrix-core kernel (gemm_f8mx.h); the launch's path is read back from the
    library's path counters."""
    from fp8_quantization_amd import _lib
    _lib.path_stats(reset=True)
    yield "f8mx"


def _ran(path):
    from fp8_quantization_amd import _lib
    st = _lib.path_stats(reset=True)
    assert st[path] >= 1 and sum(v for k, v in st.items() if k != path) == 0, st


def _all_codes(bias):
    """The 256 E4M3 values of the given bias (both zeros included)."""
    e = np.repeat(np.arange(16), 8)
    m = np.tile(np.arange(8), 16)
    v = np.where(e == 0, np.ldexp(m / 8.0, 1 - bias), np.ldexp(1.0 + m / 8.0, e - bias))
    return np.concatenate([v, -v]).astype(np.float32)


def _matmul_raw(A, B, bA, bB, bR, table, flags):
    """fp8a_matmul through ctypes with a caller-owned workspace: returns (C, flag word)."""
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
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32)) if table is not None else None
    rc = L.fp8a_matmul(_lib.dev_ptr(A), K, _lib.dev_ptr(B), N, 1, _lib.dev_ptr(C), N, Mr, N, K, 4, 3,
                       _lib.dev_ptr(tA), _lib.dev_ptr(tB), 0 if tB.numel() == 1 else 1, _lib.dev_ptr(tR),
                       _lib.host_ptr(tab) if tab is not None else None, flags, _lib.dev_ptr(ws), ws.numel(),
                       _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_matmul")
    torch.cuda.synchronize()
    flag = int(ws[:4].view(torch.int32).item())
    return C.cpu().numpy(), flag


def _terms_equal(got, ref):
    same = (got.view(np.uint32) == ref.view(np.uint32)) | ((got == 0) & (ref == 0))
    if not same.all():
        i = tuple(np.argwhere(~same)[0])
        raise AssertionError(f"{np.count_nonzero(~same)} terms differ; first at {i}: got {got[i]!r} ref {ref[i]!r}")


@pytest.mark.parametrize("table", ["nocomp", "comp", "none"])
@pytest.mark.parametrize("biases", [(12, 12, 8), (10, 13, 7), (9, 9, 2), (12, 14, 0), (8, 8, -14), (20, 18, 22)])
def test_every_code_pair_bitexact(biases, table, path):
    bA, bB, bR = biases
    A = _all_codes(bA).reshape(-1, 1)
    B = _all_codes(bB).reshape(1, -1)
    tab = gio.load("g2_matmul.npz")["E4M3_table_comp" if table == "comp" else "E4M3_table_nocomp"]
    fl = orc.flags_of(approx=table != "none", s2n=True, qbma=True)
    C, flag = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    ref = orc.terms(A, B, 4, 3, bA, bB, bR, tab, fl)[:, 0, :]
    _terms_equal(C, ref)
    # every term fits the e4m3 range of these biases: the fast form ran, nothing fell back
    assert flag == 0, "fallback flag raised: the fast form did not produce these terms"
    _ran(path)


def test_terms_beyond_e4m3_range(path):
    """Products above the result grid's top binade (Q_R lets the exponent run past max_norm, F6):
    the per-pair kernel's e4m3 conversion cannot hold them, so it flags and the exact kernel
    reruns; the one-hot path's dense terms are exact at any height -- no fallback."""
    bA, bB, bR = 12, 12, 14  # products up to ~2^7 * 3.5 exceed the result grid's top binade
    A = _all_codes(bA).reshape(-1, 1)
    B = _all_codes(bB).reshape(1, -1)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    C, flag = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    assert (flag != 0) == (path == "f8mx"), flag
    _terms_equal(C, orc.terms(A, B, 4, 3, bA, bB, bR, tab, fl)[:, 0, :])
    _ran(path)


@pytest.mark.parametrize("shape", [(256, 576, 64), (130, 300, 129), (1, 4608, 7), (512, 1152, 256)])
def test_sums_within_bar(shape, path):
    Mr, K, N = shape
    rng = np.random.default_rng(Mr + K + N)
    bA, bR = 9, 3  # no product reaches the result grid's top binade (bR <= bA + min bB - 16)
    bB = rng.integers(11, 15, size=N).astype(np.int32)
    e = rng.integers(3, 16, size=(Mr, K))
    m = rng.integers(0, 8, size=(Mr, K))
    A = np.ldexp(1.0 + m / 8.0, e - bA) * rng.choice([-1.0, 1.0], size=(Mr, K))
    A[rng.random((Mr, K)) < 0.4] = 0.0
    e = rng.integers(5, 16, size=(K, N))
    m = rng.integers(0, 8, size=(K, N))
    B = np.ldexp(1.0 + m / 8.0, e - bB[None, :]) * rng.choice([-1.0, 1.0], size=(K, N))
    A, B = A.astype(np.float32), B.astype(np.float32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    C, flag = _matmul_raw(A, B, bA, bB, bR, tab, fl)
    Cref, S = orc.matmul(A, B, 4, 3, bA, bB, bR, tab, fl, with_abs=True)
    assert flag == 0
    assert np.all(np.abs(C.astype(np.float64) - Cref) <= gio.sum_tolerance(S.astype(np.float64)))
    _ran(path)


def _sum_operands(Mr, K, N, seed):
    rng = np.random.default_rng(seed)
    bA, bR = 9, 3
    bB = rng.integers(11, 15, size=N).astype(np.int32)
    e = rng.integers(3, 16, size=(Mr, K))
    m = rng.integers(0, 8, size=(Mr, K))
    A = np.ldexp(1.0 + m / 8.0, e - bA) * rng.choice([-1.0, 1.0], size=(Mr, K))
    A[rng.random((Mr, K)) < 0.4] = 0.0
    e = rng.integers(5, 16, size=(K, N))
    m = rng.integers(0, 8, size=(K, N))
    B = np.ldexp(1.0 + m / 8.0, e - bB[None, :]) * rng.choice([-1.0, 1.0], size=(K, N))
    return A.astype(np.float32), B.astype(np.float32), bA, bB, bR


@pytest.mark.parametrize("ncg", [4, 1])
@pytest.mark.parametrize("case", ["term_out_of_range", "off_grid_a", "off_grid_b"])
def test_fallback_recomputes_only_marked_units(case, path, ncg):
    """ncg: gemm_f8mx_kernel's tile (4: 128 x 64, 1: 256 x 16 -- option "xm_ncg")."""
    from fp8_quantization_amd import _lib
    old_ncg = _lib.set_option("xm_ncg", ncg)
    try:
        _fallback_case(case, ncg)
    finally:
        _lib.set_option("xm_ncg", old_ncg)


def _fallback_case(case, ncg):
    from fp8_quantization_amd import _lib
    Mr, K, N = 520, 600, 200  # 9 x 4 output units, split-K shape
    A, B, bA, bB, bR = _sum_operands(Mr, K, N, 17)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    r, k0, n = 300, 77, 131
    if case == "term_out_of_range":  # (row k0 of B small, but for column n: the baseline stays in range)
        B[k0, :] /= 16.0
        B[k0, n] = 30.0
    C0, flag0 = _matmul_raw(A, B, bA, bB, bR, tab, fl)  # the fast path's bits, no fallback
    assert flag0 == 0
    A2, B2 = A.copy(), B.copy()
    if case == "term_out_of_range":  # on the grid (any exponent): ONE product beyond the e4m3 range of bR
        A2[r, k0] = 1024.0
    elif case == "off_grid_a":
        A2[r, k0] = 1.0 + 2.0 ** -10
    else:
        B2[k0, n] = 1.0 + 2.0 ** -12
    _lib.fallback_stats(reset=True)
    C2, flag2 = _matmul_raw(A2, B2, bA, bB, bR, tab, fl)
    st = _lib.fallback_stats()
    assert flag2 & 1 and not flag2 & 32, flag2  # some units, not all
    assert st["exact_launches"] == 1
    ur, uc = np.arange(Mr) // 64, np.arange(N) // 64
    if case == "term_out_of_range":  # the tile holding (r, n): 128 or 256 rows (gemm_f8mx_kernel's tile)
        tr = 128 if ncg == 4 else 256
        marked = ((ur[:, None] // (tr // 64)) == (r // tr)) & (uc[None, :] == n // 64)
    elif case == "off_grid_a":
        marked = (ur[:, None] == r // 64) & (uc[None, :] >= 0)
    else:
        marked = (ur[:, None] >= 0) & (uc[None, :] == n // 64)
    units = {(a, b) for a, b in zip(*np.nonzero(marked)) for a, b in [(a // 64, b // 64)]}
    assert st["exact_units"] == len(units), (st, len(units))
    # outside the marked units: the fast path's bits; inside: the exact kernel, within the bar
    same = ~marked & (np.arange(Mr)[:, None] != r)  # (row r's other outputs use the changed A element)
    assert np.array_equal(C2[same].view(np.uint32), C0[same].view(np.uint32))
    Cref, S = orc.matmul(A2, B2, 4, 3, bA, bB, bR, tab, fl, with_abs=True)
    assert np.all(np.abs(C2.astype(np.float64) - Cref) <= gio.sum_tolerance(S.astype(np.float64)))
