"""C-ABI surface checks that need no GPU: the library loads and exports every entry point
include/fp8approx.h declares; host-side argument validation reports the reference's errors."""
import ctypes
import os
import re

import pytest

from fp8_quantization_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "fp8approx.h")).read()
    return sorted(set(re.findall(r"\b(fp8a_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_match_binding_table():
    assert declared_symbols() == sorted(_lib.SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    for name in declared_symbols():
        assert hasattr(L, name), name
        assert ctypes.cast(getattr(L, name), ctypes.c_void_p).value


def test_version_string():
    assert _lib.version().startswith("fp8approx gfx950")


def _a256(x):
    return (x + 255) // 256 * 256


def _units(M, N):
    """The per-64x64-unit fallback marks after the flag word: row, column and tile bytes."""
    nur, nuc = (M + 63) // 64, (N + 63) // 64
    return _a256(nur + nuc + nur * nuc)


def _oh(M, N, K, conv_words=0, S=1):
    """The one-hot E4M3 path's buffers (gemm_oh.h): partials + correction slice, u16 A codes, B
    codes, block scales, candidate lists, count blocks (unsplit shapes: S = 1)."""
    kpad, npad = (K + 31) // 32 * 32, (N + 127) // 128 * 128
    nct = npad // 64
    aw = conv_words if conv_words else M * kpad
    return (_a256((S + 1) * M * N * 4) + _a256(aw * 2) + _a256(npad * kpad) + _a256(npad * kpad // 4) +
            _a256(kpad * nct * 256) + _a256(kpad * nct * 72))


def test_workspace_queries_are_host_only():
    L = _lib.load()
    assert L.fp8a_matmul_workspace_size() >= 4
    flag = L.fp8a_matmul_workspace_size()
    # split-K sizing is host logic (no device: 256 CUs assumed): a fraction-of-a-wave shape
    # gets room for partial sums, a many-wave shape does not; every GEMM-shaped query also
    # holds the matrix-core E4M3 path's pre-decoded operands (A words + B column pairs)
    Mr, N, K = 3211264, 64, 147
    kpad, npad = (K + 15) // 16 * 16, (N + 63) // 64 * 64
    assert L.fp8a_matmul_workspace_size_mnk(Mr, N, K) == flag + _units(Mr, N) + max(
        _a256(Mr * kpad * 4) + _a256(kpad * npad * 8) + 16384 + _a256(kpad * npad // 16 * 2), _oh(Mr, N, K))
    Mr, N, K = 12544, 512, 4608
    assert L.fp8a_matmul_workspace_size_mnk(Mr, N, K) > flag + _a256(Mr * K * 4) + _a256(K * N // 2 * 8)  # split
    # depthwise (single output channel per group): the tensor-bias kernels need the flag word and
    # the table forms' input words, + the v5 word form's (channel, tap) words
    assert L.fp8a_conv2d_workspace_size(2, 8, 6, 6, 8, 3, 3, 1, 1, 1, 1, 1, 1, 8) == flag + _a256(2 * 8 * 6 * 6 * 4) + 8 * 9 * 8
    # implicit-GEMM conv: no im2col image; the A words of one group's input slice in a zero
    # border (ph rows above / below; W % 4 == 0: a 4-word left margin and rows rounded up to 4
    # words, here 8 + 4 + 1 -> 16), + the B image (sized for the v5 form's 8 B per (k, n)) + the
    # table image + the E5M2 exponent ranges (unsplit here)
    n2 = L.fp8a_conv2d_workspace_size(2, 3, 8, 8, 4, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    assert n2 == flag + _units(2 * 8 * 8, 4) + max(_a256(2 * 3 * 10 * 16 * 4) + _a256(32 * 64 * 8) + 16384 + 256,
                                                   _oh(2 * 8 * 8, 4, 27, 2 * 3 * 10 * 16))
    n3 = L.fp8a_conv2d_workspace_size(2, 3, 7, 7, 4, 3, 3, 1, 1, 1, 1, 1, 1, 1)  # W % 4 != 0: 9 x 9
    assert n3 == flag + _units(2 * 7 * 7, 4) + max(_a256(2 * 3 * 9 * 9 * 4) + _a256(32 * 64 * 8) + 16384 + 256,
                                                   _oh(2 * 7 * 7, 4, 27, 2 * 3 * 9 * 9))
    assert L.fp8a_conv2d_workspace_size(256, 3, 224, 224, 4, 7, 7, 2, 2, 3, 3, 1, 1, 1) >= flag + 256 * 3 * 230 * 230 * 4


def test_bad_format_maps_to_value_error():
    L = _lib.load()
    rc = L.fp8a_quant(None, 0, 0, 3, None, 0, None, None)  # E = 0: rejected before any launch
    with pytest.raises(ValueError):
        _lib.check(rc, "fp8a_quant")


def test_bad_extent_maps_to_assertion_error():
    L = _lib.load()
    rc = L.fp8a_matmul(None, 2, None, 1, 1, None, 4, 3, 4, 5, 4, 3, None, None, 0, None, None, 0, None, 0, None)
    with pytest.raises(AssertionError):
        _lib.check(rc, "fp8a_matmul")


def test_word_image_queries_are_host_only():
    """fp8a_word_image_bytes / fp8a_conv2d_wants_image (the word-image hand-off,
    fp8a_conv2d_chain) are host logic: sizes of the zero-bordered image behind its 256-B header,
    and which convolutions would read one (matrix-core path with its A pre-pass: 1; the depthwise
    table form: 2)."""
    import torch
    L = _lib.load()
    # W % 4 == 0: left border widened to 4 words, rows rounded to a multiple of 4
    assert L.fp8a_word_image_bytes(2, 64, 56, 56, 1, 1) == 256 + _a256(2 * 64 * 58 * 64 * 4)
    assert L.fp8a_word_image_bytes(1, 3, 7, 7, 1, 1) == 256 + _a256(3 * 9 * 9 * 4)
    assert L.fp8a_word_image_bytes(0, 3, 7, 7, 1, 1) == 0
    fl = _lib.APPROX | _lib.S2N | _lib.QBMA
    z = torch.zeros((8, 8), dtype=torch.int32)
    z4 = torch.zeros((4, 4), dtype=torch.int32)
    wants = lambda cout, k, p, g, E, M, t, f=fl, s=1: L.fp8a_conv2d_wants_image(  # noqa: E731
        cout, k, k, p, p, g, E, M, _lib.host_ptr(t), f, s, s, 1, 1)
    assert wants(64, 3, 1, 1, 4, 3, z) == 1          # 3x3: the A pre-pass runs
    assert wants(64, 3, 1, 1, 5, 2, z4) == 1         # E5M2 too
    assert wants(64, 1, 0, 1, 4, 3, z) == 0          # 1x1, one column tile: staged from fp32
    assert wants(1024, 1, 0, 1, 4, 3, z) == 1        # 1x1, 16 column tiles: pre-pass
    assert wants(64, 3, 1, 2, 4, 3, z) == 0          # grouped
    assert wants(1, 3, 1, 1, 4, 3, z) == 0           # one output channel: tensor-bias path
    assert wants(64, 3, 1, 1, 3, 4, torch.zeros((16, 16), dtype=torch.int32)) == 0  # E3M4: tile-table kernel
    assert wants(64, 3, 1, 1, 4, 3, z, _lib.APPROX | _lib.QBMA) == 0  # no s2n: not the matrix-core form
    # single-output-channel groups (depthwise): the table form's words (form 2) only with
    # FP8A_CHAIN_TBX=1 (measured a net loss on MobileNetV2)
    tbx = 2 if os.environ.get("FP8A_CHAIN_TBX", "0") not in ("", "0") else 0
    assert wants(64, 3, 1, 64, 4, 3, z) == tbx
    assert wants(64, 3, 1, 64, 5, 2, z4, s=2) == tbx
    assert wants(64, 5, 2, 64, 4, 3, z) == 0         # 5-wide rows: the general tensor-bias kernel
    assert wants(64, 3, 1, 64, 3, 4, torch.zeros((16, 16), dtype=torch.int32)) == 0  # E3M4
