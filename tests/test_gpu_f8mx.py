"""The matrix-core E4M3 kernel (gemm_f8mx_kernel, csrc/gemm_f8mx.h).

Every case here reads the launch's flag word back and asserts it is 0, i.e. the pre-decoded,
matrix-core-summed path produced the result (not the gated exact kernel).  Biases are chosen so
every term fits the scaled e4m3 range (bA + min bB - bR >= 17: the largest term, 3.75 x
2^(30 - bA - bB), stays <= 448 x 2^(7 - bR)).  Covered:
  * implicit-GEMM conv against the oracle on unfolded inputs: ragged M / N / K, stride, padding,
    dilation, groups, split-K shapes, a 7x7 conv1-class layer;
  * the matrix form with lda > K and a column-strided B (x @ W^T as the linear layer passes it);
  * determinism (bit-identical repeats, split-K included);
  * an off-grid activation / weight / out-of-window bias raises the flag (pre-decode checks) and
    the exact kernel's result is returned;
  * a flag-only workspace still gives the right result (the VALU-accumulating form runs).
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


def _grid(rng, shape, bias, zero_frac=0.0, lo_code=3, sub_frac=0.05):
    """E4M3 values of the given bias: normal codes with expo >= lo_code, a sub_frac share of
    subnormals (m/8 * 2^(1-bias)), a zero_frac share of zeros, random signs."""
    expo = rng.integers(lo_code, 16, size=shape)
    mant = rng.integers(0, 8, size=shape)
    v = np.ldexp(1.0 + mant / 8.0, expo - bias)
    sub = rng.random(shape) < sub_frac
    v[sub] = np.ldexp(rng.integers(1, 8, size=shape) / 8.0, 1 - bias)[sub]
    v = v * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


def _tab():
    return gio.load("g2_matmul.npz")["E4M3_table_nocomp"]


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype=dtype, device=DEV)


def _conv_raw(x, w, bA, bW, bR, table, flags, stride, pad, dil, groups, ws_bytes=None):
    from fp8_quantization_amd import _lib
    L = _lib.load()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * pad - dil * (kh - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (kw - 1) - 1) // stride + 1
    xt, wt = _dev(x), _dev(w)
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=DEV)
    need = int(L.fp8a_conv2d_workspace_size(Bn, Cin, H, W, Cout, kh, kw, stride, stride, pad, pad, dil, dil, groups))
    ws = torch.zeros(need if ws_bytes is None else ws_bytes, dtype=torch.uint8, device=DEV)
    tA, tW, tR = _dev([bA], torch.int32), _dev(bW, torch.int32), _dev([bR], torch.int32)
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32))
    rc = L.fp8a_conv2d(_lib.dev_ptr(xt), _lib.dev_ptr(wt), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw, stride,
                       stride, pad, pad, dil, dil, groups, E, M, _lib.dev_ptr(tA), _lib.dev_ptr(tW), _lib.dev_ptr(tR),
                       _lib.host_ptr(tab), flags, _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_conv2d")
    torch.cuda.synchronize()
    return y.cpu().numpy(), int(ws[:4].view(torch.int32).item())


def _matmul_raw(A, lda, B, sbk, sbn, Mr, N, K, bA, bB, bR, table, flags, ws_bytes=None):
    from fp8_quantization_amd import _lib
    L = _lib.load()
    At, Bt = _dev(A), _dev(B)
    C = torch.empty((Mr, N), dtype=torch.float32, device=DEV)
    need = int(L.fp8a_matmul_workspace_size_mnk(Mr, N, K))
    ws = torch.zeros(need if ws_bytes is None else ws_bytes, dtype=torch.uint8, device=DEV)
    tA, tB, tR = _dev([bA], torch.int32), _dev(bB, torch.int32), _dev([bR], torch.int32)
    tab = torch.as_tensor(np.ascontiguousarray(table, np.int32))
    rc = L.fp8a_matmul(_lib.dev_ptr(At), lda, _lib.dev_ptr(Bt), sbk, sbn, _lib.dev_ptr(C), N, Mr, N, K, E, M,
                       _lib.dev_ptr(tA), _lib.dev_ptr(tB), 1, _lib.dev_ptr(tR), _lib.host_ptr(tab), flags,
                       _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(DEV))
    _lib.check(rc, "fp8a_matmul")
    torch.cuda.synchronize()
    return C.cpu().numpy(), int(ws[:4].view(torch.int32).item())


def _conv_ref(x, w, bA, bW, bR, table, flags, stride, pad, dil, groups):
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


def _nhwc(y):
    return y.transpose(0, 2, 3, 1).reshape(-1, y.shape[1])


def _close(got, ref, S, what=""):
    bad = np.abs(got.astype(np.float64) - ref) > gio.sum_tolerance(S.astype(np.float64))
    assert not bad.any(), f"{what}: {np.count_nonzero(bad)} outputs outside the bar"


FL = orc.flags_of(approx=True, s2n=True, qbma=True)


@pytest.mark.parametrize("cfg", [
    dict(B=2, cin=3, cout=64, k=7, s=2, p=3, d=1, g=1, hw=30),     # conv1 class, K = 147
    dict(B=3, cin=16, cout=40, k=3, s=1, p=1, d=1, g=1, hw=13),    # ragged M (507), N (40)
    dict(B=2, cin=24, cout=72, k=3, s=2, p=2, d=2, g=1, hw=17),    # dilation, N > 64
    dict(B=2, cin=32, cout=48, k=1, s=2, p=0, d=1, g=1, hw=15),    # 1x1 downsample class
    dict(B=2, cin=16, cout=32, k=3, s=1, p=1, d=1, g=2, hw=9),     # groups
    dict(B=1, cin=256, cout=128, k=3, s=1, p=1, d=1, g=1, hw=7),   # split-K (K = 2304)
    dict(B=2, cin=16, cout=24, k=3, s=2, p=1, d=1, g=1, hw=28),    # stride 2, H*W % 4 == 0 (16-B A pre-decode)
    dict(B=2, cin=24, cout=16, k=1, s=2, p=0, d=1, g=1, hw=16),    # 1x1 stride-2 downsample
    dict(B=2, cin=8, cout=20, k=3, s=2, p=2, d=2, g=2, hw=14),     # stride 2 + dilation + groups, 16-B pre-decode
    dict(B=2, cin=8, cout=20, k=3, s=2, p=2, d=2, g=2, hw=15),     # the same with H*W % 4 != 0: scalar A pre-decode
])
def test_conv_fast_path_matches_oracle(cfg):
    rng = np.random.default_rng(cfg["cin"] * 31 + cfg["cout"])
    bA, bR = 10, 7
    x = _grid(rng, (cfg["B"], cfg["cin"], cfg["hw"], cfg["hw"]), bA, zero_frac=0.45, lo_code=1)
    cig = cfg["cin"] // cfg["g"]
    bW = rng.integers(14, 17, size=cfg["cout"]).astype(np.int32)
    w = _grid(rng, (cfg["cout"], cig, cfg["k"], cfg["k"]), bW[:, None, None, None], lo_code=2)
    args = (cfg["s"], cfg["p"], cfg["d"], cfg["g"])
    y, flag = _conv_raw(x, w, bA, bW, bR, _tab(), FL, *args)
    assert flag == 0, "fallback flag raised: the matrix-core path did not produce this result"
    ref, S = _conv_ref(x, w, bA, bW, bR, _tab(), FL, *args)
    _close(_nhwc(y), ref, S, str(cfg))
    y2, _ = _conv_raw(x, w, bA, bW, bR, _tab(), FL, *args)
    assert np.array_equal(y.view(np.uint32), y2.view(np.uint32)), "not deterministic"


@pytest.mark.parametrize("shape", [(130, 300, 129), (64, 4608, 64), (257, 17, 5), (1, 64, 1)])
def test_matmul_strided_operands(shape):
    """A with lda > K, B given as W^T of a row-major [N][K] weight (sbk = 1, sbn = K)."""
    Mr, K, N = shape
    rng = np.random.default_rng(Mr + K + N)
    bA, bR = 10, 7
    lda = K + 7
    Afull = _grid(rng, (Mr, lda), bA, zero_frac=0.4)
    A = Afull[:, :K]
    bB = rng.integers(14, 17, size=N).astype(np.int32)
    W = _grid(rng, (N, K), bB[:, None])
    C, flag = _matmul_raw(Afull, lda, W, 1, K, Mr, N, K, bA, bB, bR, _tab(), FL)
    assert flag == 0
    ref, S = orc.matmul(A, W.T, E, M, bA, bB, bR, _tab(), FL, with_abs=True)
    _close(C, ref, S, str(shape))


@pytest.mark.parametrize("what", ["act", "weight", "bias"])
def test_predecode_checks_fall_back(what):
    rng = np.random.default_rng(7)
    bA, bR = 10, 7
    x = _grid(rng, (2, 16, 9, 9), bA, zero_frac=0.3)
    w = _grid(rng, (32, 16, 3, 3), 15)
    bW = np.full(32, 15, np.int32)
    if what == "act":
        x[1, 3, 4, 4] = 0.3  # off the (3, bA) grid
    elif what == "weight":
        w[5, 2, 1, 1] = 0.0123
    else:
        bW[7] = 130  # outside the exactness window of biases
    y, flag = _conv_raw(x, w, bA, bW, bR, _tab(), FL, 1, 1, 1, 1)
    assert flag != 0, "pre-decode did not flag the launch"
    ref, S = _conv_ref(x, w, bA, bW, bR, _tab(), FL, 1, 1, 1, 1)
    _close(_nhwc(y), ref, S, what)


def test_flag_only_workspace_runs_valu_form():
    rng = np.random.default_rng(11)
    bA, bR = 10, 7
    x = _grid(rng, (2, 32, 12, 12), bA, zero_frac=0.4)
    bW = rng.integers(14, 17, size=48).astype(np.int32)
    w = _grid(rng, (48, 32, 3, 3), bW[:, None, None, None])
    y, flag = _conv_raw(x, w, bA, bW, bR, _tab(), FL, 1, 1, 1, 1, ws_bytes=256)
    assert flag == 0
    ref, S = _conv_ref(x, w, bA, bW, bR, _tab(), FL, 1, 1, 1, 1)
    _close(_nhwc(y), ref, S)


def test_flag_arena_is_clean_after_a_fallback():
    """The flag word and the unit marks live in the library's per-stream flag arena, which the
    gated exact kernel leaves zero (csrc/fp8approx.hip: flag_arena, arena_release): a flagged
    launch, then clean launches of other shapes on the same stream report flag 0 and run no
    exact unit, then a flagged launch again reports its flag -- each result against the oracle."""
    from fp8_quantization_amd import _lib
    rng = np.random.default_rng(21)
    bA, bR = 10, 7
    xb = _grid(rng, (2, 16, 9, 9), bA, zero_frac=0.3)
    xb[1, 3, 4, 4] = 0.3  # off the grid: marks the second image's row units
    wb = _grid(rng, (32, 16, 3, 3), 15)
    bWb = np.full(32, 15, np.int32)
    xg = _grid(rng, (3, 16, 13, 13), bA, zero_frac=0.45, lo_code=1)
    bWg = rng.integers(14, 17, size=40).astype(np.int32)
    wg = _grid(rng, (40, 16, 3, 3), bWg[:, None, None, None], lo_code=2)
    for rep in range(2):
        _lib.fallback_stats(reset=True)
        y, flag = _conv_raw(xb, wb, bA, bWb, bR, _tab(), FL, 1, 1, 1, 1)
        assert flag != 0 and _lib.fallback_stats()["exact_units"] > 0
        ref, S = _conv_ref(xb, wb, bA, bWb, bR, _tab(), FL, 1, 1, 1, 1)
        _close(_nhwc(y), ref, S, "flagged")
        _lib.fallback_stats(reset=True)
        for _ in range(2):
            y, flag = _conv_raw(xg, wg, bA, bWg, bR, _tab(), FL, 1, 1, 1, 1)
            assert flag == 0, f"stale flag after a fallback (repeat {rep})"
            ref, S = _conv_ref(xg, wg, bA, bWg, bR, _tab(), FL, 1, 1, 1, 1)
            _close(_nhwc(y), ref, S, "clean")
        st = _lib.fallback_stats()
        assert st["exact_launches"] == 0 and st["exact_units"] == 0, st


@pytest.mark.parametrize("shape", [(300, 768, 272), (97, 100, 300), (1030, 64, 264), (3, 1024, 400)])
def test_matmul_dense_rows_predecode(shape):
    """A with lda = K % 4 == 0: the A pre-pass's 16-byte form, its (row, chunk) grid flattened over
    the launch; K not a multiple of the 64-wide K-step leaves zero words at the row ends.  N > 192:
    more than 3 column tiles, so the pre-pass runs (xm_af32)."""
    Mr, K, N = shape
    rng = np.random.default_rng(Mr * 7 + K)
    bA, bR = 10, 7
    A = _grid(rng, (Mr, K), bA, zero_frac=0.4)
    bB = rng.integers(14, 17, size=N).astype(np.int32)
    W = _grid(rng, (N, K), bB[:, None])
    C, flag = _matmul_raw(A, K, W, 1, K, Mr, N, K, bA, bB, bR, _tab(), FL)
    assert flag == 0
    ref, S = orc.matmul(A, W.T, E, M, bA, bB, bR, _tab(), FL, with_abs=True)
    _close(C, ref, S, str(shape))
    A[Mr // 2, K - 1] = 0.3  # off the grid: only that row's unit falls back
    C, flag = _matmul_raw(A, K, W, 1, K, Mr, N, K, bA, bB, bR, _tab(), FL)
    assert flag != 0
    ref, S = orc.matmul(A, W.T, E, M, bA, bB, bR, _tab(), FL, with_abs=True)
    _close(C, ref, S, str(shape) + " flagged")
