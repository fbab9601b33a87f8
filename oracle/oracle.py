"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker -- never as the thing measured or shipped.  The product path
(fp8_quantization_amd) never imports it.  Restates approx/approx_matmul_whole_v9.py of
revollllt/FP8_quantization @ 2024-11-08; see fp8approx_oracle.c for line citations.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

APPROX, S2N, QBMA, GCLIP, TB = 1, 2, 4, 8, 16
V5, OFUF, OF_OPT, UF_OPT = 32, 64, 128, 256

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I, I64, U = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint
        L.orc_decompose.argtypes = [P, I64, I, I, I, I, I, P, P]
        L.orc_quant.argtypes = [P, I64, I, I, I, I, I, P]
        L.orc_terms.argtypes = [P, I64, P, I64, P, I, I, I, I, I, I, P, I, P, U]
        L.orc_matmul.argtypes = [P, I64, P, I64, P, I64, I, I, I, I, I, I, P, I, P, U, P]
        L.orc_fp8_fake_quant.argtypes = [P, I64, I64, P, I, I, I, P, P]
        L.orc_matmul_qamaa.argtypes = [P, I64, P, I64, P, P, I, I, I, ctypes.c_float, I, I, I]
        L.orc_matmul_qamaa.restype = None
        for f in (L.orc_decompose, L.orc_quant, L.orc_terms, L.orc_matmul, L.orc_fp8_fake_quant):
            f.restype = None
        _lib = L
    return _lib


def _f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def _i32(x):
    return np.ascontiguousarray(x, dtype=np.int32)


def flags_of(approx=True, s2n=False, qbma=True, gclip=False, tb=False):
    return (APPROX if approx else 0) | (S2N if s2n else 0) | (QBMA if qbma else 0) | \
        (GCLIP if gclip else 0) | (TB if tb else 0)


def flags_v5(ofuf=False, of_opt=False, uf_opt=False):
    """v5 integer-adder model (approx_matmul_whole_v5.py) with its OF/UF switches."""
    return V5 | (OFUF if ofuf else 0) | (OF_OPT if of_opt else 0) | (UF_OPT if uf_opt else 0)


def decompose(x, E, M, b, tb=False, clip=False):
    x = _f32(x)
    e = np.empty(x.shape, np.int32)
    m = np.empty(x.shape, np.int32)
    lib().orc_decompose(x.ctypes.data, x.size, E, M, int(b), int(tb), int(clip), e.ctypes.data, m.ctypes.data)
    return e, m


def quant(x, E, M, b, tb=False, clip=False):
    x = _f32(x)
    q = np.empty(x.shape, np.float32)
    lib().orc_quant(x.ctypes.data, x.size, E, M, int(b), int(tb), int(clip), q.ctypes.data)
    return q


def _bB(bB, N):
    bB = np.asarray(bB).reshape(-1)
    if bB.size == 1:
        bB = np.repeat(bB, N)
    return _i32(bB)


def terms(A, B, E, M, bA, bB, bR, table, flags):
    A, B = _f32(A), _f32(B)
    Mr, K = A.shape
    N = B.shape[1]
    T = np.empty((Mr, K, N), np.float32)
    tab = _i32(table)
    bb = _bB(bB, N)
    lib().orc_terms(A.ctypes.data, K, B.ctypes.data, N, T.ctypes.data, Mr, N, K, E, M, int(bA),
                    bb.ctypes.data, int(bR), tab.ctypes.data, flags)
    return T


def matmul(A, B, E, M, bA, bB, bR, table, flags, with_abs=False):
    A, B = _f32(A), _f32(B)
    Mr, K = A.shape
    N = B.shape[1]
    C = np.empty((Mr, N), np.float32)
    S = np.empty((Mr, N), np.float32)
    tab = _i32(table)
    bb = _bB(bB, N)
    lib().orc_matmul(A.ctypes.data, K, B.ctypes.data, N, C.ctypes.data, N, Mr, N, K, E, M, int(bA),
                     bb.ctypes.data, int(bR), tab.ctypes.data, flags, S.ctypes.data)
    return (C, S) if with_abs else C


def fp8_fake_quant(x, maxval, E, M, per_row=False):
    x = _f32(x)
    rows = x.shape[0] if per_row else 1
    x2 = x.reshape(rows, -1)
    mx = _f32(np.asarray(maxval).reshape(-1))
    out = np.empty_like(x2)
    bias = np.empty(rows if per_row else 1, np.float32)
    lib().orc_fp8_fake_quant(x2.ctypes.data, rows, x2.shape[1], mx.ctypes.data, int(per_row), E, M,
                             out.ctypes.data, bias.ctypes.data)
    return out.reshape(x.shape), bias


def matmul_qamaa(A, B, maxval, n_bits, M, sign_bits=1):
    """(C, Cpre): fq(sum fq(a*b)) with float32 k-order sums, and the sums before the final fq."""
    A, B = _f32(A), _f32(B)
    Mr, K = A.shape
    N = B.shape[1]
    C = np.empty((Mr, N), np.float32)
    Cp = np.empty((Mr, N), np.float32)
    lib().orc_matmul_qamaa(A.ctypes.data, K, B.ctypes.data, N, C.ctypes.data, Cp.ctypes.data, Mr, N, K,
                           float(maxval), n_bits, M, sign_bits)
    return C, Cp
