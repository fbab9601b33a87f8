"""Diagnostics: does a captured launch's workspace head get zeroed on every replay?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fp8_quantization_amd import _lib, approx_ops  # noqa: E402
from fp8_quantization_amd.approx_ops import approx_conv2d, approx_matmul, make_flags  # noqa: E402
from fp8_quantization_amd.error_tables import get_error_table_NN  # noqa: E402

DEV = "cuda:0"
_lib.load()
wss = []
ws0 = approx_ops._workspace


def ws_rec(device, nbytes):
    t = ws0(device, nbytes)
    wss.append(t)
    print("ws alloc", hex(t.data_ptr()), t.numel(), flush=True)
    return t


tab = get_error_table_NN(4, 3, withComp=False, dnsmp_factor=3)
fl = make_flags(True, True, True)
g = torch.Generator().manual_seed(0)
A = torch.ldexp(torch.ones(200, 96), torch.randint(-3, 3, (200, 96))).to(DEV)
B = torch.ldexp(torch.ones(96, 72), torch.randint(-8, -4, (96, 72))).to(DEV)
bA = torch.tensor([9], dtype=torch.int32, device=DEV)
bR = torch.tensor([10], dtype=torch.int32, device=DEV)
bB = torch.full((72,), 17, dtype=torch.int32, device=DEV)
xd = torch.ldexp(torch.ones(2, 24, 10, 10), torch.randint(-3, 3, (2, 24, 10, 10))).to(DEV)
wd = torch.ldexp(torch.ones(24, 1, 3, 3), torch.randint(-8, -4, (24, 1, 3, 3))).to(DEV)
bW = torch.full((24,), 17, dtype=torch.int32, device=DEV)


def fn():
    c = approx_matmul(A, B, 4, 3, bA, bB, bR, tab, flags=fl)
    yd = approx_conv2d(xd, wd, 4, 3, bA, bW, bR, tab, flags=fl, padding=(1, 1), groups=24)
    return c, yd


gs = torch.cuda.Stream()
gs.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(gs):
    fn()
torch.cuda.current_stream().wait_stream(gs)
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
approx_ops._workspace = ws_rec
with torch.cuda.graph(gr, stream=gs, capture_error_mode="thread_local"):
    out = fn()
approx_ops._workspace = ws0
for i in range(3):
    for w in wss:
        w[:256].fill_(0xAB)
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    print("replay", i, [hex(int(w[:4].view(torch.int32).item()) & 0xFFFFFFFF) for w in wss],
          [int((w[:256] != 0).sum().item()) for w in wss], _lib.fallback_stats(reset=True), flush=True)
