"""Dense exact-product diagnostics (GPU): where outputs leave the 1e-5 sum bar."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.test_gpu_dense import _operands  # noqa: E402
from fp8_quantization_amd import _lib  # noqa: E402
from fp8_quantization_amd.approx_ops import dense_matmul  # noqa: E402

DEV = "cuda:0"
for (Mr, K, N) in [(130, 300, 129), (256, 4608, 64), (513, 64, 1000), (7, 33, 5)]:
    for fmt, (E, M) in ((0, (4, 3)), (1, (5, 2))):
        A, B = _operands(Mr, K, N, E, M, Mr + K + N + M)
        C = dense_matmul(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), fmt).cpu().numpy()
        ref = A.astype(np.float64) @ B.astype(np.float64)
        S = np.abs(A.astype(np.float64)) @ np.abs(B.astype(np.float64))
        err = np.abs(C - ref) / np.maximum(S, 1e-30)
        bad = np.argwhere(err > 1e-5)
        print((Mr, K, N), fmt, "max rel err %.3e" % err.max(), "bad", len(bad), "units", _lib.dense_stats(reset=True))
        for (m, n) in bad[:4]:
            prods = A[m].astype(np.float64) * B[:, n]
            print("   m", m, "n", n, "C", C[m, n], "ref", ref[m, n], "S", S[m, n], "diff", C[m, n] - ref[m, n])
            # which 32-k blocks: the diff vs partial sums omitting one product
            d = C[m, n] - ref[m, n]
            close = np.argsort(np.abs(prods + d))[:3]
            print("   products closest to -diff:", [(int(k), prods[k], A[m, k], B[k, n]) for k in close])
            blk = [float(np.abs(A[m, 32 * b:32 * b + 32]).max()) for b in range((K + 31) // 32)]
            print("   A row block maxima", blk[:12])
            bb = [float(np.abs(B[32 * b:32 * b + 32, n]).max()) for b in range((K + 31) // 32)]
            print("   B col block maxima", bb[:12])
