"""Pin the CPU oracle against vectors produced by the reference itself (tests/golden).

Bit-exact on decompose fields, Q_R values and every per-product term; sums within the
summation-order tolerance of SURVEY §8(d).
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tests import golden_io as gio

META = gio.meta()


@pytest.mark.parametrize("case", META["g1"], ids=lambda c: c["key"])
def test_g1_decompose_and_quant_bitexact(case):
    g = gio.load("g1_decompose.npz")
    key, E, M, b = case["key"], case["E"], case["M"], case["b"]
    x = g[key + "_x"]
    for tb in (0, 1):
        for clip in (0, 1):
            sfx = f"_tb{tb}_c{clip}"
            e, m = orc.decompose(x, E, M, b, tb=tb, clip=clip)
            q = orc.quant(x, E, M, b, tb=tb, clip=clip)
            np.testing.assert_array_equal(e, g[key + sfx + "_expo"], err_msg=key + sfx)
            np.testing.assert_array_equal(m, g[key + sfx + "_mant"], err_msg=key + sfx)
            np.testing.assert_array_equal(q.view(np.uint32), g[key + sfx + "_q"].view(np.uint32),
                                          err_msg=key + sfx)


def _table(g2, fmt, tname):
    return g2[f"{fmt}_table_{tname}"]


@pytest.mark.parametrize("case", META["g2"], ids=lambda c: c["key"])
def test_g2_terms_bitexact_and_sums(case):
    g = gio.load("g2_matmul.npz")
    fmt, key = case["fmt"], case["key"]
    A, B = g[fmt + "_A"], g[fmt + "_B"]
    tab = _table(g, fmt, case["table"])
    fl = gio.flags_from(case)
    T = orc.terms(A[:8, :64], B[:64, :8], case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl)
    ref_T = g[key + "_T"]
    np.testing.assert_array_equal(T.view(np.uint32) & 0x7FFFFFFF | 0, ref_T.view(np.uint32) & 0x7FFFFFFF,
                                  err_msg="term magnitudes")
    nz = ref_T != 0
    np.testing.assert_array_equal(np.signbit(T[nz]), np.signbit(ref_T[nz]), err_msg="term signs")
    C, S = orc.matmul(A[:64], B[:, :64], case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl,
                      with_abs=True)
    ref_C = g[key + "_C"]
    assert np.all(np.abs(C - ref_C) <= gio.sum_tolerance(S)), np.max(np.abs(C - ref_C) / (S + 1e-30))


@pytest.mark.parametrize("case", META["g3"], ids=lambda c: c["key"])
def test_g3_debug_params_layer(case):
    g = gio.load("g3_debug.npz")
    g2 = gio.load("g2_matmul.npz")
    tab = _table(g2, "E3M4", case["table"])
    bB = g["bB"].astype(np.int32)
    C, S = orc.matmul(g["A"], g["B"], 3, 4, int(g["bA"][0]), bB, int(g["bR"][0]), tab, gio.flags_from(case),
                      with_abs=True)
    ref = g[case["key"] + "_C"]
    assert np.all(np.abs(C - ref) <= gio.sum_tolerance(S))


@pytest.mark.parametrize("case", META["g4"], ids=lambda c: c["key"])
def test_g4_tensor_bias_terms_bitexact(case):
    g = gio.load("g4_tensorbias.npz")
    g2 = gio.load("g2_matmul.npz")
    fmt, key = case["fmt"], case["key"]
    A, B = g[fmt + "_A"], g[fmt + "_B"]
    tab = _table(g2, fmt, case["table"])
    fl = gio.flags_from(case, tb=True)
    T = orc.terms(A, B, case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl)
    ref_T = g[key + "_T"]
    np.testing.assert_array_equal(np.abs(T), np.abs(ref_T))
    C, S = orc.matmul(A, B, case["E"], case["M"], case["bA"], case["bB"], case["bR"], tab, fl, with_abs=True)
    assert np.all(np.abs(C - g[key + "_C"]) <= gio.sum_tolerance(S))


@pytest.mark.parametrize("case", META["g6"], ids=lambda c: c["key"])
def test_g6_qamaa(case):
    """qamaa vs the reference: identical wherever the pre-quantisation sums agree; where the
    reference's torch sum order and the k-order sum straddle an FP8 rounding boundary the
    outputs may differ by one FP8 step (both are correct roundings of sums equal within
    fp32 summation error)."""
    g = gio.load("g6_qamaa.npz")
    A, B = g[case["fmt"] + "_A"], g[case["fmt"] + "_B"]
    C, Cpre = orc.matmul_qamaa(A, B, case["maxval"], 8, case["M"])
    ref = g[case["key"] + "_C"]
    diff = C != ref
    assert diff.mean() < 0.02, diff.mean()
    if diff.any():
        step = np.ldexp(1.0, np.floor(np.log2(np.abs(ref[diff]) + 1e-30)).astype(int) - case["M"])
        assert np.all(np.abs(C[diff] - ref[diff]) <= step * 1.0001)


@pytest.mark.parametrize("case", META["g7"], ids=lambda c: c["key"])
def test_g7_v5_integer_adder_terms_bitexact_and_sums(case):
    """v5 integer-adder model with sim_hw_add_OFUF / with_OF_opt / with_UF_opt (SURVEY §8(f)
    next-4): per-product terms bit-exact, sums within the accumulation tolerance."""
    g = gio.load("g7_v5.npz")
    A, B, tab, fl = gio.v5_case(case)
    E, M, b = case["E"], case["M"], case["bias"]
    T = orc.terms(A[:6], B[:, :6], E, M, b, b, b, tab, fl)
    Tr = g[case["key"] + "_T"]
    same = (T.view(np.uint32) == Tr.view(np.uint32)) | ((T == 0) & (Tr == 0))
    assert same.all(), f"{np.count_nonzero(~same)} terms differ"
    C, S = orc.matmul(A, B, E, M, b, b, b, tab, fl, with_abs=True)
    assert np.all(np.abs(C.astype(np.float64) - g[case["key"] + "_C"]) <= gio.sum_tolerance(S))
