"""gemm_tt_kernel<5> with the band / zero wave-tile forms on and off (option tt_band), on a ResNet-50
3x3-layer-shaped product at three result biases: every product in the band, all below half the
quantum, and the realistic mix; milliseconds per launch (HIP events)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fp8_quantization_amd import _lib  # noqa: E402
from fp8_quantization_amd.approx_ops import approx_matmul, make_flags  # noqa: E402
from fp8_quantization_amd.error_tables import get_error_table_NN  # noqa: E402

DEV = "cuda:0"
_lib.load()
E, M = 2, 5
rng = np.random.default_rng(0)


def grid(shape, bias, zf):
    expo = rng.integers(1, 4, size=shape)
    mant = rng.integers(0, 32, size=shape)
    v = np.ldexp(1.0 + mant / 32.0, expo - bias) * rng.choice([-1.0, 1.0], size=shape)
    v[rng.random(shape) < zf] = 0
    return torch.from_numpy(v.astype(np.float32)).to(DEV)


Mr, K, N = 25088, 2304, 256
bA, bB = 4, 9
A = grid((Mr, K), bA, 0.4)
B = grid((K, N), bB, 0.0)
tab = get_error_table_NN(E, M, withComp=False, dnsmp_factor=3)
fl = make_flags(True, True, True)
tA = torch.tensor([bA], dtype=torch.int32, device=DEV)
tB = torch.full((N,), bB, dtype=torch.int32, device=DEV)
top = 4 - bA + 4 - bB
for name, bR in (("band", 1 - top), ("zero", -top - M), ("mixed", bA + 1)):
    tR = torch.tensor([bR], dtype=torch.int32, device=DEV)
    for opt in (0, 1):
        _lib.set_option("tt_band", opt)
        for _ in range(2):
            C = approx_matmul(A, B, E, M, tA, tB, tR, tab, flags=fl)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            C = approx_matmul(A, B, E, M, tA, tB, tR, tab, flags=fl)
        b.record()
        torch.cuda.synchronize()
        print(f"{name:6s} bR={bR:4d} tt_band={opt}: {a.elapsed_time(b) / 5:.3f} ms  "
              f"{2 * Mr * K * N / (a.elapsed_time(b) / 5e3) / 1e12:.2f} TFLOP/s", flush=True)
_lib.set_option("tt_band", 1)
