"""ctypes binding of libfp8approx.so (the gfx950 HIP library; C-ABI in include/fp8approx.h).

There is no CPU or PyTorch fallback: if the library is missing or cannot be loaded, every
entry point raises.  Device work needs HIP tensors; CPU tensors are rejected.
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FP8A_LIB_PATH") or os.path.join(HERE, "lib", "libfp8approx.so")

APPROX, S2N, QBMA, GCLIP, TB = 1, 2, 4, 8, 16
V5, OFUF, OF_OPT, UF_OPT = 32, 64, 128, 256  # v5 integer-adder model (include/fp8approx.h)
OK, EINVAL, EFORMAT, EHIP = 0, -1, -2, -3
DENSE_E4M3, DENSE_E5M2, DENSE_BF16 = 0, 1, 2  # fp8a_dense_* operand formats

SYMBOLS = ("fp8a_version", "fp8a_last_error", "fp8a_fallback_stats", "fp8a_path_stats", "fp8a_kernel_timing", "fp8a_kernel_time", "fp8a_set_option", "fp8a_decompose", "fp8a_quant", "fp8a_matmul_workspace_size",
           "fp8a_matmul_workspace_size_mnk", "fp8a_matmul", "fp8a_terms", "fp8a_conv2d_workspace_size", "fp8a_conv2d",
           "fp8a_conv2d_bn_act", "fp8a_conv2d_qin_workspace_size", "fp8a_conv2d_qin",
           "fp8a_conv2d_block_workspace_size", "fp8a_conv2d_block", "fp8a_max_pool2d", "fp8a_avg_pool2d_plane", "fp8a_im2col",
           "fp8a_fp8_quantize", "fp8a_matmul_qamaa", "fp8a_conv2d_qamaa", "fp8a_matmul_block_workspace_size",
           "fp8a_matmul_block", "fp8a_dense_matmul_workspace_size", "fp8a_dense_matmul",
           "fp8a_dense_conv2d_workspace_size", "fp8a_dense_conv2d", "fp8a_grouped_conv2d", "fp8a_dense_conv2d_fused", "fp8a_dense_stats", "fp8a_clock_stats",
           "fp8a_word_image_bytes", "fp8a_word_image_init", "fp8a_conv2d_chain", "fp8a_conv2d_wants_image",
           "fp8a_flag_arena_slot_bytes")

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes handle; raise if the HIP library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} not found: build it with `python -m fp8_quantization_amd.build_native` "
            "(there is no CPU fallback for the approx-FP8 path)")
    L = ctypes.CDLL(LIB_PATH)
    P, I, I64, U, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, ctypes.c_size_t
    F = ctypes.c_float
    sig = {
        "fp8a_version": ([], ctypes.c_char_p),
        "fp8a_last_error": ([], ctypes.c_char_p),
        "fp8a_fallback_stats": ([P, I], I),
        "fp8a_path_stats": ([P, I], I),
        "fp8a_kernel_timing": ([I], I),
        "fp8a_kernel_time": ([P, I], I),
        "fp8a_set_option": ([ctypes.c_char_p, I], I),
        "fp8a_decompose": ([P, I64, I64, I64, I, I, P, I64, U, P, P, P], I),
        "fp8a_quant": ([P, I64, I, I, P, U, P, P], I),
        "fp8a_matmul_workspace_size": ([], SZ),
        "fp8a_matmul_workspace_size_mnk": ([I64, I64, I64], SZ),
        "fp8a_matmul": ([P, I64, P, I64, I64, P, I64, I64, I64, I64, I, I, P, P, I64, P, P, U, P, SZ, P], I),
        "fp8a_terms": ([P, I64, P, I64, I64, P, I64, I64, I64, I, I, P, P, I64, P, P, U, P], I),
        "fp8a_conv2d_workspace_size": ([I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I], SZ),
        "fp8a_conv2d": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P, U, P, SZ, P],
                        I),
        "fp8a_conv2d_bn_act": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P, U, P,
                                I, F, F, P, SZ, P], I),
        "fp8a_conv2d_qin_workspace_size": ([I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I], SZ),
        "fp8a_conv2d_qin": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, I, I, P, P, P, U, P, I, F,
                             F, P, I, I, I, P, P, P, SZ, P], I),
        "fp8a_conv2d_block_workspace_size": ([I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I], SZ),
        "fp8a_conv2d_block": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P, U, P, I,
                               F, F, P, I, I, I, P, P, P, I, F, F, P, I, I, I, P, P, P, SZ, P], I),
        "fp8a_word_image_bytes": ([I64, I64, I64, I64, I, I], SZ),
        "fp8a_word_image_init": ([P, I64, I64, I64, I64, I, I, P], I),
        "fp8a_conv2d_wants_image": ([I64, I, I, I, I, I, I, I, P, U, I, I, I, I], I),
        "fp8a_conv2d_chain": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P, U, P, I,
                               F, F, P, I, I, I, P, P, P, I, F, F, P, I, I, I, P, P, P, P, I, I, P, I, I, I, P, I,
                               I, P, SZ, P], I),
        "fp8a_max_pool2d": ([P, P, I64, I64, I64, I64, I, I, I, I, I, I, P], I),
        "fp8a_avg_pool2d_plane": ([P, P, I64, I64, I64, I64, I, I, I, I, P], I),
        "fp8a_im2col": ([P, P, I64, I64, I64, I64, I, I, I, I, I, I, I, I, P], I),
        "fp8a_fp8_quantize": ([P, I64, I64, P, I, I, I, I, P, P, P, P], I),
        "fp8a_matmul_qamaa": ([P, I64, P, I64, I64, P, I64, I64, I64, P, I, I, I, P], I),
        "fp8a_conv2d_qamaa": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, P, I, I, I, P], I),
        "fp8a_matmul_block_workspace_size": ([I64, I64, I64], SZ),
        "fp8a_matmul_block": ([P, I64, P, I64, I64, P, I64, I64, I64, I64, I, I, P, P, I64, P, P, U, P, I, F, F, P, I, I,
                               I, P, P, P, I, F, F, P, I, I, I, P, P, P, SZ, P], I),
        "fp8a_dense_matmul_workspace_size": ([I64, I64, I64], SZ),
        "fp8a_dense_matmul": ([P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, I, P, SZ, P], I),
        "fp8a_dense_conv2d_workspace_size": ([I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I], SZ),
        "fp8a_dense_conv2d": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, P, SZ, P], I),
        "fp8a_grouped_conv2d": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, P], I),
        "fp8a_dense_conv2d_fused": ([P, P, P, I64, I64, I64, I64, I64, I, I, I, I, I, I, I, I, I, I,
                                     P, I, I, I, I, P, P, P, I, I, I, P, P, P, I, I, I, P, P, P, I, F, F,
                                     P, I, I, I, P, P, P, SZ, P], I),
        "fp8a_dense_stats": ([P, I], I),
        "fp8a_clock_stats": ([P, I], I),
        "fp8a_flag_arena_slot_bytes": ([P], SZ),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def version():
    return load().fp8a_version().decode()


def check(rc, what):
    """Map a C-ABI return code onto the reference's exception types."""
    if rc == OK:
        return
    msg = f"{what}: {load().fp8a_last_error().decode()}"
    if rc == EINVAL:
        raise AssertionError(msg)      # approx_matmul_whole_v9.py:20
    if rc == EFORMAT:
        raise ValueError(msg)          # approx_matmul_whole_v9.py:590
    raise RuntimeError(msg)


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def dev_ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("fp8approx kernels need HIP device tensors (no CPU fallback)")
    return ctypes.c_void_p(t.data_ptr())


def host_ptr(t):
    assert t.device.type == "cpu" and t.is_contiguous()
    return ctypes.c_void_p(t.data_ptr())


def flag_arena_slot_bytes(device=None):
    """fp8a_flag_arena_slot_bytes of the current stream of `device` (0 before its first eager launch)."""
    return int(load().fp8a_flag_arena_slot_bytes(stream_ptr(device)))


def fallback_stats(reset=False):
    """fp8a_fallback_stats: dict(exact_launches, exact_units, f32_reruns, tb_launches) since load /
    the last reset (synchronises the device)."""
    L = load()
    out = (ctypes.c_uint64 * 4)()
    check(L.fp8a_fallback_stats(ctypes.cast(out, ctypes.c_void_p), 1 if reset else 0), "fp8a_fallback_stats")
    return dict(exact_launches=int(out[0]), exact_units=int(out[1]), f32_reruns=int(out[2]), tb_launches=int(out[3]))


PATHS = ("f8mx", "tt", "tt16", "fast", "exact", "dense", "v5mx")


def path_stats(reset=False):
    """fp8a_path_stats: launches per GEMM path since load / the last reset."""
    L = load()
    out = (ctypes.c_uint64 * len(PATHS))()
    check(L.fp8a_path_stats(ctypes.cast(out, ctypes.c_void_p), 1 if reset else 0), "fp8a_path_stats")
    return {k: int(v) for k, v in zip(PATHS, out)}


def kernel_timing(enable):
    """fp8a_kernel_timing: record HIP events around every GEMM's product kernel; returns the
    previous state."""
    return int(load().fp8a_kernel_timing(1 if enable else 0))


def kernel_time(reset=False):
    """fp8a_kernel_time: {path: dict(ms, launches, dispatches, macs)} of the recorded launches
    (synchronises on their events)."""
    L = load()
    out = (ctypes.c_double * (4 * len(PATHS)))()
    check(L.fp8a_kernel_time(ctypes.cast(out, ctypes.c_void_p), 1 if reset else 0), "fp8a_kernel_time")
    return {k: dict(ms=out[4 * i], launches=int(out[4 * i + 1]), dispatches=int(out[4 * i + 2]), macs=out[4 * i + 3])
            for i, k in enumerate(PATHS) if out[4 * i + 1] > 0}


_option_gen = 0


def option_generation():
    """Incremented by every set_option call (caches of option-dependent host decisions key on it)."""
    return _option_gen


def set_option(name, value):
    """fp8a_set_option: returns the previous value."""
    global _option_gen
    rc = load().fp8a_set_option(name.encode(), int(value))
    if rc < 0:
        check(rc, "fp8a_set_option")
    _option_gen += 1
    return rc


def dense_stats(reset=False):
    """fp8a_dense_stats: dict(fp32_launches, fp32_units) -- dense exact-product launches with
    64 x 64 units recomputed in fp32, and those units (synchronises the device)."""
    L = load()
    out = (ctypes.c_uint64 * 2)()
    check(L.fp8a_dense_stats(ctypes.cast(out, ctypes.c_void_p), 1 if reset else 0), "fp8a_dense_stats")
    return dict(fp32_launches=int(out[0]), fp32_units=int(out[1]))


def clock_stats(reset=False):
    """fp8a_clock_stats (a -DFP8A_CLOCK_STAMP=1 build): dict(memtime, realtime, workgroups, ghz)."""
    L = load()
    out = (ctypes.c_uint64 * 3)()
    check(L.fp8a_clock_stats(ctypes.cast(out, ctypes.c_void_p), 1 if reset else 0), "fp8a_clock_stats")
    t, r, n = int(out[0]), int(out[1]), int(out[2])
    return dict(memtime=t, realtime=r, workgroups=n, ghz=(t / r * 0.1) if r else None)
