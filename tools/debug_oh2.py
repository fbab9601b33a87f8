"""Debug probe 2: correction on/off at K = 4, and the correction slice alone vs the true corrections."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle as orc  # noqa: E402
from tests import golden_io as gio  # noqa: E402
from tests.test_gpu_f8 import _matmul_raw, _sum_operands  # noqa: E402
from fp8_quantization_amd import _lib  # noqa: E402

tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
fl = orc.flags_of(approx=True, s2n=True, qbma=True)
_lib.set_option("one_hot", 1)
for K in (3, 4):
    A, B, bA, bB, bR = _sum_operands(128, K, 128, 3)
    # dense check with scales uniform: put every weight of a column in the same binade
    ref, S = orc.matmul(A, B, 4, 3, bA, bB, bR, tab, fl, with_abs=True)
    for corr in (1, 0):
        _lib.set_option("oh_correct", corr)
        C, flag = _matmul_raw(A, B, bA, bB, bR, tab, fl)
        err = np.abs(C.astype(np.float64) - ref) / (S + 1e-30)
        i = np.unravel_index(np.argmax(err), err.shape)
        print(f"K={K} correct={corr} max_rel={err.max():.3g} at {i}: got {C[i]} ref {ref[i]} S {S[i]}", flush=True)
        if K == 4 and corr == 1:
            T = orc.terms(A[i[0]:i[0]+1], B[:, i[1]:i[1]+1], 4, 3, bA, bB, bR, tab, fl)[0, :, 0]
            print("  terms", T, "A", A[i[0]], "B", B[:, i[1]], "bB", bB[i[1]])
_lib.set_option("oh_correct", 1)
