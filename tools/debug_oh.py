"""Debug probe for the one-hot E4M3 path (gemm_oh.h): max error vs the oracle over K (GPU)."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as orc  # noqa: E402
from tests import golden_io as gio  # noqa: E402
from tests.test_gpu_f8 import _matmul_raw, _sum_operands  # noqa: E402
from fp8_quantization_amd import _lib  # noqa: E402

tab = gio.load("g2_matmul.npz")["E4M3_table_nocomp"]
fl = orc.flags_of(approx=True, s2n=True, qbma=True)
for path in ("one_hot", "f8mx"):
    _lib.set_option("one_hot", path == "one_hot")
    for K in (1, 2, 4, 5, 8, 16, 17, 32, 33, 64, 576):
      for bRx in (None, 40):
        for (Mr, N) in ((256, 64), (128, 128)):
            A, B, bA, bB, bR = _sum_operands(Mr, K, N, 3)
            if bRx is not None:
                bR = bRx  # no candidate pairs: the dense part alone
            if len(sys.argv) > 1 and sys.argv[1] == "uniform":
                bB[:] = bB[0]
                A, B, bA, bB, bR = A, B, bA, bB, bR
            C, flag = _matmul_raw(A, B, bA, bB, bR, tab, fl)
            ref, S = orc.matmul(A, B, 4, 3, bA, bB, bR, tab, fl, with_abs=True)
            err = np.abs(C.astype(np.float64) - ref) / (S.astype(np.float64) + 1e-30)
            bad = err > 1e-5
            print(f"{path:8s} K={K:4d} bR={bR} M={Mr} N={N} flag={flag} max_rel={err.max():.3g} bad={bad.sum()}"
                  f" bad_rows={np.unique(np.nonzero(bad)[0])[:8]} bad_cols={np.unique(np.nonzero(bad)[1])[:8]}",
                  flush=True)
print(_lib.path_stats())
