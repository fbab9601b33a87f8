"""Accumulation behaviour of the block-scaled MFMA as dn_gemm uses it (GPU): rows of A probe how
far below the largest product a product still lands exactly, within one 32-k block and across
blocks (different block scales), B = 1.0."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from fp8_quantization_amd import _lib  # noqa: E402
from fp8_quantization_amd.approx_ops import dense_matmul  # noqa: E402

DEV = "cuda:0"
K, N = 128, 16
rows, names = [], []
for e in range(1, 31):
    r = np.zeros(K); r[0] = 1.0; r[40] = 2.0 ** -e; rows.append(r); names.append(f"1 + 2^-{e} (k 40, block 1)")
for e in range(1, 18):
    r = np.zeros(K); r[0] = 1.0; r[1] = 2.0 ** -e; rows.append(r); names.append(f"1 + 2^-{e} (k 1, same block)")
for e in range(2, 30, 2):
    r = np.zeros(K); r[0] = 1.0; r[32:96] = 2.0 ** -e; rows.append(r); names.append(f"1 + 64 x 2^-{e} (blocks 1-2)")
for e in range(2, 20, 2):
    r = np.zeros(K); r[0] = 1.0; r[1:32] = 2.0 ** -e; rows.append(r); names.append(f"1 + 31 x 2^-{e} (block 0)")
for e in range(2, 30, 2):
    r = np.zeros(K); r[40] = 1.0; r[0] = 2.0 ** -e; rows.append(r); names.append(f"2^-{e} (k 0) + 1 (k 40)")
A = np.array(rows, np.float32)
B = np.ones((K, N), np.float32)
_lib.dense_stats(reset=True)
C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), _lib.DENSE_E4M3).cpu().numpy()
print("fp32 units", _lib.dense_stats(reset=True))
ex = A.astype(np.float64).sum(1)
for i, nm in enumerate(names):
    print("%-32s D=%.10g exact=%.10g err/ulp(exact)=%g" % (nm, C[i, 0], ex[i], (C[i, 0] - ex[i]) / np.spacing(np.float32(ex[i]))))
