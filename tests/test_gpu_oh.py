"""The E4M3 one-hot path (csrc/gemm_oh.h): a dense e4m3 x bf8 matrix-core GEMM over K' = 8K plus
the exact correction of the candidate pairs (products below the result grid's smallest normal,
and weights excluded from their MX block's window).

Checked against the CPU oracle (the reference's term restated, tests/golden pins it):
  * realistic operands (ReLU activations and Gaussian weights through the FP8 quantizer, biases
    from the quantizer as the hijacker sets them) over ragged shapes, with bR chosen so that a few
    percent of the products are candidates: sums within 1e-5 sum|term|, no fallback, the one-hot
    path ran;
  * single-term outputs (A one-hot along K, so every output is one term plus exact zeros) over
    K = 4 blocks whose weights span more than the block window (excluded weights), the subnormal
    band and the flush-to-zero region: bit-exact;
  * split-K shapes: within the bar and bit-identical from run to run (the correction's LDS float
    atomics included).
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
    old = _lib.set_option("one_hot", 1)
    yield
    _lib.set_option("one_hot", old)


def _quant(x, per_row=False):
    mx = np.abs(x).max(axis=1) if per_row else np.abs(x).max()
    q, b = orc.fp8_fake_quant(x, np.maximum(mx, 1e-30), 4, 3, per_row=per_row)
    return q.astype(np.float32), np.rint(b).astype(np.int32)


def _operands(Mr, K, N, seed, spread=1.0):
    rng = np.random.default_rng(seed)
    A, bA = _quant(np.maximum(rng.standard_normal((Mr, K)), 0.0).astype(np.float32))
    W = (rng.standard_normal((N, K)) * 0.05 * np.exp(rng.standard_normal((N, 1)) * spread)).astype(np.float32)
    Wq, bB = _quant(W, per_row=True)
    return A, np.ascontiguousarray(Wq.T), int(bA[0]), bB.reshape(-1)


def _run(A, B, bA, bB, bR, tab, fl):
    from tests.test_gpu_f8 import _matmul_raw
    return _matmul_raw(A, B, bA, bB, bR, tab, fl)


def _check_path():
    from fp8_quantization_amd import _lib
    st = _lib.path_stats(reset=True)
    assert st["one_hot"] >= 1 and st["f8mx"] == 0, st


@pytest.mark.parametrize("table", ["nocomp", "comp"])
@pytest.mark.parametrize("shape", [(256, 576, 64), (130, 300, 129), (1, 4608, 7), (512, 1152, 256), (77, 33, 200),
                                   (1000, 147, 64)])
def test_sums_realistic_operands(shape, table):
    from fp8_quantization_amd import _lib
    Mr, K, N = shape
    A, B, bA, bB = _operands(Mr, K, N, sum(shape))
    # the result quantizer's bias from the largest exact sum (as calibration would set it)
    bR = int(np.rint(15 - np.log2(np.abs(A.astype(np.float64) @ B).max() + 1e-30) + np.log2(1.875) - 1))
    tab = gio.load("g2_matmul.npz")["E4M3_table_" + table]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    _lib.path_stats(reset=True)
    C, flag = _run(A, B, bA, bB, bR, tab, fl)
    _check_path()
    Cref, S = orc.matmul(A, B, 4, 3, bA, bB, bR, tab, fl, with_abs=True)
    assert flag == 0, flag
    bad = np.abs(C.astype(np.float64) - Cref) > gio.sum_tolerance(S.astype(np.float64))
    assert not bad.any(), f"{bad.sum()} outputs outside the bar"
    # the candidates are a real part of the workload, not an empty set
    T = orc.terms(A[:8], B, 4, 3, bA, bB, bR, tab, fl)
    prod = np.abs(A[:8, :, None].astype(np.float64) * B[None].astype(np.float64))
    assert np.count_nonzero((prod > 0) & (prod < 2.0 ** (1 - bR))) > 0 or Mr * K < 64


@pytest.mark.parametrize("bR", [4, 10, 13, 16])
def test_single_terms_bitexact_with_excluded_weights(bR):
    """Every output is ONE term (A has a single nonzero per row, at k = row % K): the dense term
    plus the correction must be the reference's term exactly, including weights more than 12
    binades below their 4-k block's largest (excluded from the MX block: dense term 0, the
    correction supplies the whole term) and products in / below the subnormal band."""
    from fp8_quantization_amd import _lib
    rng = np.random.default_rng(bR)
    K, N, bA = 8, 96, 10
    bB = rng.integers(14, 20, size=N).astype(np.int32)
    e = np.arange(1, 16)
    # A: every E4M3 code of bias bA over the rows, one nonzero per row
    ea = np.repeat(e, 8)
    ma = np.tile(np.arange(8), 15)
    vals = np.ldexp(1.0 + ma / 8.0, ea - bA)
    vals = np.concatenate([vals, -vals, np.ldexp(np.arange(1, 8) / 8.0, 1 - bA)])  # + subnormal codes
    Mr = vals.size
    A = np.zeros((Mr, K), np.float32)
    A[np.arange(Mr), np.arange(Mr) % K] = vals
    # B: per 4-k block one large weight and three spread over 20 binades below it
    eb = rng.integers(0, 16, size=(K, N))
    big = (np.arange(K) % 4 == 0)[:, None]
    eb = np.where(big, 15, rng.integers(0, 16, size=(K, N)))
    mb = rng.integers(0, 8, size=(K, N))
    B = np.where(eb == 0, np.ldexp(mb / 8.0, 1 - bB[None, :]), np.ldexp(1.0 + mb / 8.0, eb - bB[None, :]))
    B = (B * rng.choice([-1.0, 1.0], size=(K, N))).astype(np.float32)
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    _lib.path_stats(reset=True)
    C, flag = _run(A, B, bA, bB, bR, tab, fl)
    _check_path()
    assert flag == 0, flag
    T = orc.terms(A, B, 4, 3, bA, bB, bR, tab, fl)
    ref = T[np.arange(Mr), np.arange(Mr) % K, :]
    same = (C.view(np.uint32) == ref.view(np.uint32)) | ((C == 0) & (ref == 0))
    assert same.all(), f"{np.count_nonzero(~same)} terms differ; first {np.argwhere(~same)[0]}"


@pytest.mark.parametrize("shape", [(256, 4608, 64), (96, 2304, 256)])
def test_split_k_within_bar_and_deterministic(shape):
    from fp8_quantization_amd import _lib
    Mr, K, N = shape
    A, B, bA, bB = _operands(Mr, K, N, 5)
    bR = int(np.rint(15 - np.log2(np.abs(A.astype(np.float64) @ B).max() + 1e-30)))
    tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
    fl = orc.flags_of(approx=True, s2n=True, qbma=True)
    _lib.path_stats(reset=True)
    C1, f1 = _run(A, B, bA, bB, bR, tab, fl)
    C2, f2 = _run(A, B, bA, bB, bR, tab, fl)
    _check_path()
    assert f1 == 0 and f2 == 0
    assert np.array_equal(C1.view(np.uint32), C2.view(np.uint32)), "run-to-run results differ"
    Cref, S = orc.matmul(A, B, 4, 3, bA, bB, bR, tab, fl, with_abs=True)
    assert np.all(np.abs(C1.astype(np.float64) - Cref) <= gio.sum_tolerance(S.astype(np.float64)))
