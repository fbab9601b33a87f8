"""One v5 E5M2 K = 1 product through fp8a_matmul (the first gemm_v5mx_kernel launch of
tests/test_gpu_v5.py::test_g7_v5_terms_and_sums[E5M2_b15_zero_s100]), synchronised after every
launch (HIP_LAUNCH_BLOCKING) -- diagnostic only."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from fp8_quantization_amd import _lib  # noqa: E402
from fp8_quantization_amd.approx_v5 import custom_matmul_vectorize  # noqa: E402

A = np.ldexp(1.0 + np.arange(6).reshape(6, 1) % 4 / 4.0, -np.arange(6).reshape(6, 1)).astype(np.float32)
B = np.ldexp(1.0 + np.arange(6).reshape(1, 6) % 4 / 4.0, np.arange(6).reshape(1, 6) - 3).astype(np.float32)
tab = torch.zeros(4, 4, dtype=torch.int32)
print("paths before", _lib.path_stats(reset=True), flush=True)
C = custom_matmul_vectorize(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(), 5, 2, None, tab,
                            sim_hw_add_OFUF=True)
torch.cuda.synchronize()
print("paths", _lib.path_stats(reset=True), flush=True)
print(C.cpu().numpy(), flush=True)
