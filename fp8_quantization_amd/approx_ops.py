"""Host side of the approx_v9 hot path: torch custom ops over the gfx950 C-ABI.

Mirrors the reference module approx/approx_matmul_whole_v9.py (revollllt/FP8_quantization
@ 2024-11-08): ``custom_matmul_vectorize`` keeps its signature and argument meaning
(v9:10-18), ``quant_to_fp_any_vectorize_torch`` (v9:333) and ``float_to_fpany_absint_torch``
(v9:233, here taking (E, M, bias) instead of a param dict) are the element codecs,
``get_error_table_NN`` the table selection (v9:555).  All arithmetic runs in
libfp8approx.so; these wrappers only marshal pointers, biases and flags.

Bias typing follows the reference: Python ints select the int-bias semantics, int tensors the
tensor-bias semantics (quirk F5 -- param_prepare's integer powers flush min_norm to 0), which
is what approx_multiply passes for single-column products (approx_calculation.py:800-809).
"""
import ctypes
import os
from typing import Optional

import torch
from torch import nn

from . import _lib
from .error_tables import get_error_table_NN  # noqa: F401  (re-exported, v9:555)

__all__ = ["custom_matmul_vectorize", "approx_matmul", "approx_matmul_block", "approx_terms", "approx_conv2d", "qamaa_matmul", "qamaa_conv2d",
           "quant_to_fp_any_vectorize_torch", "float_to_fpany_absint_torch", "get_error_table_NN",
           "make_flags", "make_flags_v5", "fp8_fake_quantize", "bn_act_epilogue", "dense_format", "dense_matmul",
           "dense_conv2d", "grouped_conv2d", "dense_conv2d_fused"]


def make_flags(with_approx=True, with_s2nn2s_opt=False, quant_btw_mult_accu=True, golden_clip_OF=False,
               tensor_bias=False):
    return ((_lib.APPROX if with_approx else 0) | (_lib.S2N if with_s2nn2s_opt else 0) |
            (_lib.QBMA if quant_btw_mult_accu else 0) | (_lib.GCLIP if golden_clip_OF else 0) |
            (_lib.TB if tensor_bias else 0))


def make_flags_v5(sim_hw_add_OFUF=False, with_OF_opt=False, with_UF_opt=False):
    """Flags of the v5 integer-adder model (approx_matmul_whole_v5.py:155-183)."""
    return (_lib.V5 | (_lib.OFUF if sim_hw_add_OFUF else 0) | (_lib.OF_OPT if with_OF_opt else 0) |
            (_lib.UF_OPT if with_UF_opt else 0))


def _uses_table(flags):
    return bool(flags & (_lib.APPROX | _lib.V5))


_BIAS_CACHE = {}

# bench.py sets this to a list to time every approx launch with HIP events on the current
# stream: entries (start_event, end_event, approx_MACs).  None = no instrumentation.
_PROFILE = None


def _prof_start():
    if _PROFILE is None:
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _prof_end(start, macs, nbytes=0):
    """nbytes: the launch's algorithmic HBM bytes (operands read once, output written once), for
    the memory-bound dense exact product; 0 for the approx ops (priced by MACs)."""
    if start is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        _PROFILE.append((start, ev, int(macs), int(nbytes)))


def _bias_dev(b, device, n=None):
    """Device int32 bias vector from an int or a (float/int) tensor; no host sync for tensors."""
    if isinstance(b, torch.Tensor):
        i32 = getattr(b, "_fp8a_i32", None)  # set by fp8_fake_quantize: no conversion launch
        if i32 is not None and i32.device == device:
            return i32
        t = b.detach().reshape(-1)
        if t.device != device:
            t = t.to(device)
        if t.dtype != torch.int32:
            t = t.to(torch.int32)  # float biases are torch.round() outputs: exact
        return t.contiguous()
    key = (device, int(b))
    t = _BIAS_CACHE.get(key)
    if t is None:
        t = torch.tensor([int(b)], dtype=torch.int32, device=device)
        _BIAS_CACHE[key] = t
    return t


def _table_host(error_table_NN, mant_width, with_approx):
    n = 2 ** mant_width
    if error_table_NN is None or not with_approx:
        return torch.zeros((n, n), dtype=torch.int32)
    t = error_table_NN.detach()
    if t.device.type != "cpu" or t.dtype != torch.int32 or not t.is_contiguous():
        t = t.to(device="cpu", dtype=torch.int32).contiguous()  # host table: packed into kernargs
    if t.shape != (n, n):
        raise AssertionError(f"error table must be {n}x{n}, got {tuple(t.shape)}")
    return t


def _workspace(device, nbytes):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def _as_f32(x):
    if x.dtype != torch.float32:
        x = x.float()
    return x


# ----------------------------------------------------------------------------------- matmul
@torch.library.custom_op("fp8approx::matmul", mutates_args=())
def _matmul_op(A: torch.Tensor, B: torch.Tensor, bA: torch.Tensor, bB: torch.Tensor, bR: torch.Tensor,
               table: torch.Tensor, E: int, M: int, flags: int) -> torch.Tensor:
    L = _lib.load()
    dev = A.device
    if not A.is_contiguous() and A.stride(1) != 1:
        A = A.contiguous()
    Mr, K = A.shape
    N = B.shape[1]
    C = torch.empty((Mr, N), dtype=torch.float32, device=dev)
    ws = _workspace(dev, L.fp8a_matmul_workspace_size_mnk(Mr, N, K))
    bBs = 0 if bB.numel() == 1 else 1
    rc = L.fp8a_matmul(_lib.dev_ptr(A), A.stride(0), _lib.dev_ptr(B), B.stride(0), B.stride(1),
                       _lib.dev_ptr(C), N, Mr, N, K, E, M, _lib.dev_ptr(bA), _lib.dev_ptr(bB), bBs,
                       _lib.dev_ptr(bR), _lib.host_ptr(table), flags, _lib.dev_ptr(ws), ws.numel(),
                       _lib.stream_ptr(dev))
    _lib.check(rc, "fp8a_matmul")
    return C


@_matmul_op.register_fake
def _(A, B, bA, bB, bR, table, E, M, flags):
    return A.new_empty((A.shape[0], B.shape[1]), dtype=torch.float32)


def approx_matmul(A, B, E, M, bA, bB, bR, table=None, flags=None, **flag_kwargs):
    """C[m, n] = sum_k approx_v9 term(A[m, k], B[k, n]) on the GPU.

    A [M, K] and B [K, N] float32 device tensors (any strides with a unit stride dimension;
    weight.t() views are consumed in place).  bB: int, 1-element or per-column [N] tensor.
    """
    if A.dim() != 2 or B.dim() != 2 or A.shape[1] != B.shape[0]:
        raise AssertionError(f"approx_matmul: shape mismatch {tuple(A.shape)} @ {tuple(B.shape)}")  # v9:20
    if flags is None:
        flags = make_flags(**flag_kwargs)
    A, B = _as_f32(A), _as_f32(B)
    if B.stride(0) != 1 and B.stride(1) != 1:
        B = B.contiguous()
    dev = A.device
    tab = _table_host(table, M, _uses_table(flags))
    bB_ = _bias_dev(bB, dev)
    if bB_.numel() not in (1, B.shape[1]):
        raise AssertionError(f"approx_matmul: {bB_.numel()} column biases for {B.shape[1]} columns")
    ev = _prof_start()
    C = _matmul_op(A, B, _bias_dev(bA, dev), bB_, _bias_dev(bR, dev), tab, int(E), int(M), int(flags))
    _prof_end(ev, A.shape[0] * A.shape[1] * B.shape[1])
    return C


@torch.library.custom_op("fp8approx::matmul_block", mutates_args=())
def _matmul_block_op(A: torch.Tensor, B: torch.Tensor, bA: Optional[torch.Tensor], bB: torch.Tensor,
                     bR: torch.Tensor, table: torch.Tensor, E: int, M: int, flags: int, bn: Optional[torch.Tensor],
                     in_maxval: Optional[torch.Tensor], in_nbits: int, in_mbits: int, in_sign_bits: int,
                     res: Optional[torch.Tensor], post_act: int, post_lo: float, post_hi: float,
                     out_maxval: Optional[torch.Tensor], out_nbits: int, out_mbits: int, out_sign_bits: int
                     ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """fp8a_matmul_block: C = fq_out(clamp(bn(fq_in(A) @ B) + res)); returns C and the input /
    output quantizers' float and int32 biases (1-element tensors, unset when unused)."""
    L = _lib.load()
    dev = A.device
    A = A.contiguous()
    Mr, K = A.shape
    N = B.shape[1]
    C = torch.empty((Mr, N), dtype=torch.float32, device=dev)
    ib, iib = torch.empty(1, device=dev), torch.empty(1, dtype=torch.int32, device=dev)
    ob, oib = torch.empty(1, device=dev), torch.empty(1, dtype=torch.int32, device=dev)
    if res is not None:
        res = res.contiguous()
        if res.shape != C.shape or res.dtype != torch.float32 or res.device != dev:
            raise AssertionError(f"approx_matmul_block: residual must be float32 {tuple(C.shape)} on {dev}")
    if bn is not None and (bn.shape != (N, 2) or bn.dtype != torch.float32 or not bn.is_contiguous()):
        raise AssertionError(f"approx_matmul_block: epilogue parameters must be contiguous float32 [{N}, 2]")
    ws = _workspace(dev, L.fp8a_matmul_block_workspace_size(Mr, N, K))
    opt = lambda t: _lib.dev_ptr(t) if t is not None else None  # noqa: E731
    rc = L.fp8a_matmul_block(_lib.dev_ptr(A), K, _lib.dev_ptr(B), B.stride(0), B.stride(1), _lib.dev_ptr(C), N, Mr,
                             N, K, E, M, opt(bA), _lib.dev_ptr(bB), 0 if bB.numel() == 1 else 1, _lib.dev_ptr(bR),
                             _lib.host_ptr(table), flags, opt(bn), 0, 0.0, 0.0, opt(in_maxval), int(in_nbits),
                             int(in_mbits), int(in_sign_bits), _lib.dev_ptr(ib), _lib.dev_ptr(iib), opt(res),
                             int(post_act), float(post_lo), float(post_hi), opt(out_maxval), int(out_nbits),
                             int(out_mbits), int(out_sign_bits), _lib.dev_ptr(ob), _lib.dev_ptr(oib), _lib.dev_ptr(ws),
                             ws.numel(), _lib.stream_ptr(dev))
    _lib.check(rc, "fp8a_matmul_block")
    return C, ib, iib, ob, oib


@_matmul_block_op.register_fake
def _(A, B, bA, bB, bR, table, E, M, flags, bn, in_maxval, in_nbits, in_mbits, in_sign_bits, res, post_act, post_lo,
      post_hi, out_maxval, out_nbits, out_mbits, out_sign_bits):
    one = A.new_empty((1,))
    onei = A.new_empty((1,), dtype=torch.int32)
    return A.new_empty((A.shape[0], B.shape[1])), one, onei, one.clone(), onei.clone()


def bias_epilogue(bias, device):
    """The store epilogue {1, bias} per column for a linear's bias: x * 1 + bias is exactly the
    reference's ``out += bias``."""
    with torch.no_grad():
        b = _as_f32(bias.detach()).reshape(-1).to(device)
        return torch.stack((torch.ones_like(b), b), dim=1).contiguous()


def approx_matmul_block(A, B, E, M, bA, bB, bR, table=None, flags=None, bias=None, qin=None, post=None,
                        bias_epi=None):
    """approx_matmul with the linear layer's neighbours fused into the same launch:
    C = fq_out(clamp(fq_in(A) @ B + bias + residual)).

    bias: the linear's bias [N] or None (applied as the store's x * 1 + bias, i.e. exactly the
    reference's ``out += bias``); bias_epi: the same as a prebuilt ``bias_epilogue`` tensor.  qin / post: as approx_conv2d (per-tensor quantizer tuples; A is
    then UNQUANTIZED and bA unused).  Returns ``(C, input quantizer bias or None, output quantizer
    bias or None)``."""
    if A.dim() != 2 or B.dim() != 2 or A.shape[1] != B.shape[0]:
        raise AssertionError(f"approx_matmul: shape mismatch {tuple(A.shape)} @ {tuple(B.shape)}")  # v9:20
    A, B = _as_f32(A), _as_f32(B)
    if B.stride(0) != 1 and B.stride(1) != 1:
        B = B.contiguous()
    dev = A.device
    tab = _table_host(table, M, _uses_table(flags))
    bB_ = _bias_dev(bB, dev)
    if bB_.numel() not in (1, B.shape[1]):
        raise AssertionError(f"approx_matmul: {bB_.numel()} column biases for {B.shape[1]} columns")
    bn = bias_epi if bias_epi is not None else (bias_epilogue(bias, dev) if bias is not None else None)
    iq = _quantizer_args(qin) if qin is not None else (None, 0, 0, 0)
    res, pact, plo, phi, oq = post if post is not None else (None, 0, 0.0, 0.0, None)
    oq = _quantizer_args(oq) if oq is not None else (None, 0, 0, 0)
    ev = _prof_start()
    C, ib, iib, ob, oib = _matmul_block_op(
        A, B, None if qin is not None else _bias_dev(bA, dev), bB_, _bias_dev(bR, dev), tab, int(E), int(M),
        int(flags), bn, iq[0].to(dev) if iq[0] is not None else None, iq[1], iq[2], iq[3],
        _as_f32(res) if res is not None else None, int(pact), float(plo), float(phi),
        oq[0].to(dev) if oq[0] is not None else None, oq[1], oq[2], oq[3])
    _prof_end(ev, A.shape[0] * A.shape[1] * B.shape[1])
    ib._fp8a_i32 = iib
    ob._fp8a_i32 = oib
    return C, (ib if qin is not None else None), (ob if oq[0] is not None else None)


def approx_terms(A, B, E, M, bA, bB, bR, table=None, flags=None, **flag_kwargs):
    """Per-product terms T[m, k, n] (the values the reference sums at v9:113); parity tool."""
    if A.shape[1] != B.shape[0]:
        raise AssertionError("approx_terms: inner dimensions differ")
    if flags is None:
        flags = make_flags(**flag_kwargs)
    L = _lib.load()
    A, B = _as_f32(A), _as_f32(B)
    dev = A.device
    Mr, K = A.shape
    N = B.shape[1]
    T = torch.empty((Mr, K, N), dtype=torch.float32, device=dev)
    bA_, bB_, bR_ = _bias_dev(bA, dev), _bias_dev(bB, dev), _bias_dev(bR, dev)
    tab = _table_host(table, M, _uses_table(flags))
    rc = L.fp8a_terms(_lib.dev_ptr(A), A.stride(0), _lib.dev_ptr(B), B.stride(0), B.stride(1), _lib.dev_ptr(T),
                      Mr, N, K, int(E), int(M), _lib.dev_ptr(bA_), _lib.dev_ptr(bB_), 0 if bB_.numel() == 1 else 1,
                      _lib.dev_ptr(bR_), _lib.host_ptr(tab), int(flags), _lib.stream_ptr(dev))
    _lib.check(rc, "fp8a_terms")
    return T


def custom_matmul_vectorize(A, B, expo_width, mant_width, custom_bias_A, custom_bias_B, custom_bias_R,
                            error_table_NN, with_approx=True, with_s2nn2s_opt=False, sim_hw_add_OFUF=False,
                            with_OF_opt=False, with_UF_opt=False, golden_clip_OF=False, quant_btw_mult_accu=True,
                            debug_mode=False, self_check_mode=False):
    """Drop-in for approx_matmul_whole_v9.custom_matmul_vectorize (v9:10-169).

    sim_hw_add_OFUF / with_OF_opt / with_UF_opt are accepted and ignored, as in v9.
    """
    assert A.shape[1] == B.shape[0]
    tb = [isinstance(b, torch.Tensor) for b in (custom_bias_A, custom_bias_B, custom_bias_R)]
    if any(tb) and not all(tb):
        raise NotImplementedError("mixed int / tensor biases: pass all three the same way")
    flags = make_flags(with_approx, with_s2nn2s_opt, quant_btw_mult_accu, golden_clip_OF, tensor_bias=all(tb))
    out = approx_matmul(A, B, expo_width, mant_width, custom_bias_A, custom_bias_B, custom_bias_R,
                        error_table_NN, flags=flags)
    if self_check_mode:
        golden = quant_to_fp_any_vectorize_torch(A.unsqueeze(2) * B.unsqueeze(0), expo_width, mant_width,
                                                 custom_bias_R, clip_OF=golden_clip_OF) \
            if quant_btw_mult_accu else A.unsqueeze(2) * B.unsqueeze(0)
        err = (golden.sum(dim=1) - out).abs()
        print("\n====== Self-Checking Mode ======")
        print(f"MatMul Max  Error     : {err.max()}")
        print(f"MatMul Mean Error     : {err.mean()}")
        print(f"MatMul RMSE           : {torch.sqrt(torch.mean(err ** 2))}")
    return out


# ----------------------------------------------------------------------------------- codecs
def _codec_bias(custom_bias, device):
    if custom_bias is None:
        raise NotImplementedError("pass the bias explicitly")
    return _bias_dev(custom_bias, device), isinstance(custom_bias, torch.Tensor)


def quant_to_fp_any_vectorize_torch(arr, expo_width, mant_width, custom_bias=None, clip_OF=True):
    """Q_R (v9:333-362) on the GPU.  custom_bias None means the IEEE-style default 2^(E-1)-1."""
    if custom_bias is None:
        custom_bias = 2 ** (expo_width - 1) - 1
    L = _lib.load()
    x = _as_f32(arr).contiguous()
    b, tb = _codec_bias(custom_bias, x.device)
    out = torch.empty_like(x)
    rc = L.fp8a_quant(_lib.dev_ptr(x), x.numel(), int(expo_width), int(mant_width), _lib.dev_ptr(b),
                      make_flags(False, False, False, clip_OF, tb), _lib.dev_ptr(out), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_quant")
    return out


def float_to_fpany_absint_torch(values, expo_width, mant_width, custom_bias, clip_OF=False):
    """DEC (v9:233-291): returns (expo, mant) int32 tensors shaped like values."""
    L = _lib.load()
    x = _as_f32(values).contiguous()
    b, tb = _codec_bias(custom_bias, x.device)
    e = torch.empty(x.shape, dtype=torch.int32, device=x.device)
    m = torch.empty_like(e)
    rc = L.fp8a_decompose(_lib.dev_ptr(x), 1, x.numel(), x.numel(), int(expo_width), int(mant_width),
                          _lib.dev_ptr(b), 0, make_flags(False, False, False, clip_OF, tb), _lib.dev_ptr(e),
                          _lib.dev_ptr(m), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_decompose")
    return e, m


# ----------------------------------------------------------------------------------- conv
@torch.library.custom_op("fp8approx::conv2d", mutates_args=())
def _conv2d_op(x: torch.Tensor, w: torch.Tensor, bA: torch.Tensor, bW: torch.Tensor, bR: torch.Tensor,
               table: torch.Tensor, E: int, M: int, flags: int, stride: list[int], padding: list[int],
               dilation: list[int], groups: int, bn: Optional[torch.Tensor] = None, act: int = 0,
               act_lo: float = 0.0, act_hi: float = 0.0) -> torch.Tensor:
    L = _lib.load()
    x = x.contiguous()
    w = w.contiguous()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    Ho = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    Wo = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    nbytes = L.fp8a_conv2d_workspace_size(Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, groups)
    ws = _workspace(x.device, nbytes)
    if bn is None:
        rc = L.fp8a_conv2d(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw, sh, sw,
                           ph, pw, dh, dw, groups, E, M, _lib.dev_ptr(bA), _lib.dev_ptr(bW), _lib.dev_ptr(bR),
                           _lib.host_ptr(table), flags, _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(x.device))
        _lib.check(rc, "fp8a_conv2d")
        return y
    if bn.shape != (Cout, 2) or bn.dtype != torch.float32 or not bn.is_contiguous() or bn.device != x.device:
        raise AssertionError(f"approx_conv2d: epilogue parameters must be contiguous float32 [{Cout}, 2] "
                             f"on {x.device}, got {tuple(bn.shape)} {bn.dtype} on {bn.device}")
    rc = L.fp8a_conv2d_bn_act(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw, sh, sw,
                              ph, pw, dh, dw, groups, E, M, _lib.dev_ptr(bA), _lib.dev_ptr(bW), _lib.dev_ptr(bR),
                              _lib.host_ptr(table), flags, _lib.dev_ptr(bn), int(act), float(act_lo), float(act_hi),
                              _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_conv2d_bn_act")
    return y


@_conv2d_op.register_fake
def _(x, w, bA, bW, bR, table, E, M, flags, stride, padding, dilation, groups, bn=None, act=0, act_lo=0.0,
      act_hi=0.0):
    Bn, _, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    return x.new_empty((Bn, Cout, Ho, Wo))


@torch.library.custom_op("fp8approx::conv2d_block", mutates_args=())
def _conv2d_block_op(x: torch.Tensor, w: torch.Tensor, bA: Optional[torch.Tensor], bW: torch.Tensor,
                     bR: torch.Tensor, table: torch.Tensor, E: int, M: int, flags: int, stride: list[int],
                     padding: list[int], dilation: list[int], groups: int, in_maxval: Optional[torch.Tensor],
                     in_nbits: int, in_mbits: int, in_sign_bits: int, res: Optional[torch.Tensor], post_act: int,
                     post_lo: float, post_hi: float, out_maxval: Optional[torch.Tensor], out_nbits: int,
                     out_mbits: int, out_sign_bits: int, bn: Optional[torch.Tensor] = None, act: int = 0,
                     act_lo: float = 0.0, act_hi: float = 0.0
                     ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """fp8a_conv2d_block: y = fq_out(clamp(bn_act(conv(fq_in(x))) + res)); returns y and the input /
    output quantizers' float and int32 biases (1-element tensors, unset when unused)."""
    L = _lib.load()
    x = x.contiguous()
    w = w.contiguous()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    Ho = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    Wo = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    ib, iib = torch.empty(1, device=x.device), torch.empty(1, dtype=torch.int32, device=x.device)
    ob, oib = torch.empty(1, device=x.device), torch.empty(1, dtype=torch.int32, device=x.device)
    if res is not None:
        res = res.contiguous()
        if res.shape != y.shape or res.dtype != torch.float32 or res.device != x.device:
            raise AssertionError(f"approx_conv2d: residual must be float32 {tuple(y.shape)} on {x.device}")
    if bn is not None and (bn.shape != (Cout, 2) or bn.dtype != torch.float32 or not bn.is_contiguous()):
        raise AssertionError(f"approx_conv2d: epilogue parameters must be contiguous float32 [{Cout}, 2]")
    ws = _workspace(x.device, L.fp8a_conv2d_block_workspace_size(Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh,
                                                                 dw, groups))
    opt = lambda t: _lib.dev_ptr(t) if t is not None else None  # noqa: E731
    rc = L.fp8a_conv2d_block(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw, sh, sw,
                             ph, pw, dh, dw, groups, E, M, opt(bA), _lib.dev_ptr(bW), _lib.dev_ptr(bR),
                             _lib.host_ptr(table), flags, opt(bn), int(act), float(act_lo), float(act_hi),
                             opt(in_maxval), int(in_nbits), int(in_mbits), int(in_sign_bits), _lib.dev_ptr(ib),
                             _lib.dev_ptr(iib), opt(res), int(post_act), float(post_lo), float(post_hi),
                             opt(out_maxval), int(out_nbits), int(out_mbits), int(out_sign_bits), _lib.dev_ptr(ob),
                             _lib.dev_ptr(oib), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_conv2d_block")
    return y, ib, iib, ob, oib


@_conv2d_block_op.register_fake
def _(x, w, bA, bW, bR, table, E, M, flags, stride, padding, dilation, groups, in_maxval, in_nbits, in_mbits,
      in_sign_bits, res, post_act, post_lo, post_hi, out_maxval, out_nbits, out_mbits, out_sign_bits, bn=None, act=0,
      act_lo=0.0, act_hi=0.0):
    Bn, _, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    one = x.new_empty((1,))
    onei = x.new_empty((1,), dtype=torch.int32)
    return x.new_empty((Bn, Cout, Ho, Wo)), one, onei, one.clone(), onei.clone()


# in_image is mutated too: an image that arrived invalid is re-decoded in place by the consumer's
# gated pre-pass (xm_decode_a / tbx_decode_a write its words from x)
@torch.library.custom_op("fp8approx::conv2d_chain", mutates_args=("in_image", "out_image"))
def _conv2d_chain_op(x: torch.Tensor, w: torch.Tensor, bA: Optional[torch.Tensor], bW: torch.Tensor,
                     bR: torch.Tensor, table: torch.Tensor, E: int, M: int, flags: int, stride: list[int],
                     padding: list[int], dilation: list[int], groups: int, in_maxval: Optional[torch.Tensor],
                     in_nbits: int, in_mbits: int, in_sign_bits: int, res: Optional[torch.Tensor], post_act: int,
                     post_lo: float, post_hi: float, out_maxval: Optional[torch.Tensor], out_nbits: int,
                     out_mbits: int, out_sign_bits: int, in_image: Optional[torch.Tensor],
                     out_image: Optional[torch.Tensor], next_ph: int, next_pw: int,
                     next_maxval: Optional[torch.Tensor], next_nbits: int, next_mbits: int, next_sign_bits: int,
                     next_bR: Optional[torch.Tensor], next_Mw: int, bn: Optional[torch.Tensor] = None, act: int = 0,
                     act_lo: float = 0.0, act_hi: float = 0.0, next_form: int = 0
                     ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """fp8a_conv2d_chain: fp8a_conv2d_block that reads its input's word image (in_image) and / or
    emits the next convolution's (out_image); same results and return values as conv2d_block."""
    L = _lib.load()
    x = x.contiguous()
    w = w.contiguous()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    Ho = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    Wo = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    ib, iib = torch.empty(1, device=x.device), torch.empty(1, dtype=torch.int32, device=x.device)
    ob, oib = torch.empty(1, device=x.device), torch.empty(1, dtype=torch.int32, device=x.device)
    if res is not None:
        res = res.contiguous()
        if res.shape != y.shape or res.dtype != torch.float32 or res.device != x.device:
            raise AssertionError(f"approx_conv2d: residual must be float32 {tuple(y.shape)} on {x.device}")
    if bn is not None and (bn.shape != (Cout, 2) or bn.dtype != torch.float32 or not bn.is_contiguous()):
        raise AssertionError(f"approx_conv2d: epilogue parameters must be contiguous float32 [{Cout}, 2]")
    # (a single-output-channel-group consumer reads table-form words: an image without border)
    in_pad = (ph, pw) if groups == 1 else (0, 0)
    # (form 1, the table form, has no border; forms 0 and 2 -- matrix-core and v5 words -- carry the
    # consumer's padding, as fp8a_conv2d_chain sizes them)
    out_pad = (0, 0) if next_form == 1 else (next_ph, next_pw)
    for img, shp in ((in_image, (Bn, Cin, H, W) + in_pad), (out_image, (Bn, Cout, Ho, Wo) + out_pad)):
        if img is not None and img.numel() < L.fp8a_word_image_bytes(*shp):
            raise AssertionError("approx_conv2d: word image smaller than fp8a_word_image_bytes")
    ws = _workspace(x.device, L.fp8a_conv2d_block_workspace_size(Bn, Cin, H, W, Cout, kh, kw, sh, sw, ph, pw, dh,
                                                                 dw, groups))
    opt = lambda t: _lib.dev_ptr(t) if t is not None else None  # noqa: E731
    rc = L.fp8a_conv2d_chain(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw, sh, sw,
                             ph, pw, dh, dw, groups, E, M, opt(bA), _lib.dev_ptr(bW), _lib.dev_ptr(bR),
                             _lib.host_ptr(table), flags, opt(bn), int(act), float(act_lo), float(act_hi),
                             opt(in_maxval), int(in_nbits), int(in_mbits), int(in_sign_bits), _lib.dev_ptr(ib),
                             _lib.dev_ptr(iib), opt(res), int(post_act), float(post_lo), float(post_hi),
                             opt(out_maxval), int(out_nbits), int(out_mbits), int(out_sign_bits), _lib.dev_ptr(ob),
                             _lib.dev_ptr(oib), opt(in_image), opt(out_image), int(next_ph), int(next_pw),
                             opt(next_maxval), int(next_nbits), int(next_mbits), int(next_sign_bits), opt(next_bR),
                             int(next_Mw), int(next_form), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_conv2d_chain")
    return y, ib, iib, ob, oib


@_conv2d_chain_op.register_fake
def _(x, w, bA, bW, bR, table, E, M, flags, stride, padding, dilation, groups, in_maxval, in_nbits, in_mbits,
      in_sign_bits, res, post_act, post_lo, post_hi, out_maxval, out_nbits, out_mbits, out_sign_bits, in_image,
      out_image, next_ph, next_pw, next_maxval, next_nbits, next_mbits, next_sign_bits, next_bR, next_Mw, bn=None,
      act=0, act_lo=0.0, act_hi=0.0, next_form=0):
    Bn, _, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    one = x.new_empty((1,))
    onei = x.new_empty((1,), dtype=torch.int32)
    return x.new_empty((Bn, Cout, Ho, Wo)), one, onei, one.clone(), onei.clone()


def word_image_bytes(Bn, C, H, W, ph, pw):
    """fp8a_word_image_bytes: bytes of a convolution input's word image (0: bad arguments)."""
    return int(_lib.load().fp8a_word_image_bytes(int(Bn), int(C), int(H), int(W), int(ph), int(pw)))


def new_word_image(Bn, C, H, W, ph, pw, device):
    """A freshly initialised word image (fp8a_word_image_init) for a convolution input of shape
    [Bn, C, H, W] and padding (ph, pw): a 256-byte aligned uint8 device tensor."""
    n = word_image_bytes(Bn, C, H, W, ph, pw)
    if n == 0:
        raise AssertionError("new_word_image: bad shape")
    buf = torch.empty(n + 256, dtype=torch.uint8, device=device)
    off = (-buf.data_ptr()) % 256
    img = buf[off:off + n]
    rc = _lib.load().fp8a_word_image_init(_lib.dev_ptr(img), int(Bn), int(C), int(H), int(W), int(ph), int(pw),
                                          _lib.stream_ptr(torch.device(device)))
    _lib.check(rc, "fp8a_word_image_init")
    return img


def conv2d_wants_image(Cout, kernel, padding, groups, E, M, table, flags, stride=(1, 1), dilation=(1, 1)):
    """fp8a_conv2d_wants_image: the input word image a convolution would read -- 0 none, 1 the
    matrix-core form (image of its padding), 2 the tensor-bias table form (image without border)."""
    tab = _table_host(table, M, _uses_table(flags))
    return int(_lib.load().fp8a_conv2d_wants_image(int(Cout), int(kernel[0]), int(kernel[1]), int(padding[0]),
                                                   int(padding[1]), int(groups), int(E), int(M),
                                                   _lib.host_ptr(tab), int(flags) & ~_lib.TB, int(stride[0]),
                                                   int(stride[1]), int(dilation[0]), int(dilation[1])))


def _quantizer_args(q):
    """(maxval [1] device tensor, n_bits, mantissa bits, sign bits) of a per-tensor quantizer tuple."""
    mx, nb, mb, sb = q
    mx = _as_f32(mx).reshape(-1).contiguous()
    if mx.numel() != 1:
        raise AssertionError("approx_conv2d: fused quantizers must be per tensor")
    return mx, int(nb), int(mb), int(sb)


def approx_conv2d(x, w, E, M, bA, bW, bR, table=None, flags=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1),
                  groups=1, epilogue=None, qin=None, post=None, chain=None, **flag_kwargs):
    """approx_v9 convolution, NCHW in / NCHW out (pre-BN), K ordered (c, ky, kx) like the
    reference im2col (approx_calculation.py:724-747); single-output-channel groups get the
    tensor-bias semantics (approx_calculation.py:800-809).  bW: per output channel.

    epilogue: optional ``(scale_shift [Cout, 2] float32 device tensor, act, lo, hi)`` fusing
    the layer's eval-mode BatchNorm (y * scale + shift) and a clamp activation into the
    kernel's store (fp8a_conv2d_bn_act, include/fp8approx.h); see ``bn_act_epilogue``.

    qin: optional ``(maxval [1] device tensor, n_bits, mantissa_bits, sign_bits)`` of the layer's
    per-tensor input activation quantizer: x is then UNQUANTIZED, the op applies
    quantize_to_fp8_ste_MM itself (fp8a_conv2d_qin: inside the E4M3 operand pre-decode where that
    path runs); bA is unused.

    post: optional ``(residual tensor or None, clamp (0/1), lo, hi, output quantizer tuple or
    None)``: a residual block's tail in the store, y = fq_out(clamp(y + residual))
    (fp8a_conv2d_block).

    chain: optional ``(in_image or None, out or None)`` -- the word-image hand-off
    (fp8a_conv2d_chain): in_image is x's word image emitted by the previous convolution (needs
    qin); out = ``(image, next padding (ph, pw), next input quantizer tuple, next result bias
    [1] int32 device tensor, next mantissa width)`` emits the next convolution's.  Bit-identical
    results; x / y are still read / written as fp32.

    With qin, post or chain the result is ``(y, input quantizer bias or None, output quantizer bias
    or None)`` -- the float biases the quantizers would have set as their custom_bias."""
    if flags is None:
        flags = make_flags(**flag_kwargs)
    flags &= ~_lib.TB
    dev = x.device
    tab = _table_host(table, M, _uses_table(flags))
    bW_ = _bias_dev(bW, dev)
    if bW_.numel() == 1:
        bW_ = bW_.expand(w.shape[0]).contiguous()
    if bW_.numel() != w.shape[0]:
        raise AssertionError(f"approx_conv2d: {bW_.numel()} weight biases for {w.shape[0]} output channels")
    ev = _prof_start()
    if chain is not None:
        iq = _quantizer_args(qin) if qin is not None else (None, 0, 0, 0)
        res, pact, plo, phi, oq = post if post is not None else (None, 0, 0.0, 0.0, None)
        oq = _quantizer_args(oq) if oq is not None else (None, 0, 0, 0)
        in_img, out = chain
        if in_img is not None and qin is None:
            raise AssertionError("approx_conv2d: an input word image needs the fused input quantizer")
        if out is not None:
            oimg, (nph, npw), nq, nbR, nM = out[:5]
            nform = out[5] if len(out) > 5 else 0
            nq = _quantizer_args(nq)
            nbR = _bias_dev(nbR, dev)
        else:
            oimg, nph, npw, nq, nbR, nM, nform = None, 0, 0, (None, 0, 0, 0), None, 0, 0
        y, ib, iib, ob, oib = _conv2d_chain_op(
            _as_f32(x), _as_f32(w), None if qin is not None else _bias_dev(bA, dev), bW_, _bias_dev(bR, dev), tab,
            int(E), int(M), int(flags), [int(s) for s in stride], [int(p) for p in padding],
            [int(d) for d in dilation], int(groups), iq[0].to(dev) if iq[0] is not None else None, iq[1], iq[2],
            iq[3], res, int(pact), float(plo), float(phi), oq[0].to(dev) if oq[0] is not None else None, oq[1],
            oq[2], oq[3], in_img, oimg, int(nph), int(npw), nq[0].to(dev) if nq[0] is not None else None, nq[1],
            nq[2], nq[3], nbR, int(nM), *(epilogue or ()), next_form=int(nform))
        ib._fp8a_i32 = iib
        ob._fp8a_i32 = oib
        _prof_end(ev, y.shape[0] * y.shape[2] * y.shape[3] * w.shape[0] * w.shape[1] * w.shape[2] * w.shape[3])
        return y, (ib if qin is not None else None), (ob if oq[0] is not None else None)
    if qin is not None or post is not None:
        iq = _quantizer_args(qin) if qin is not None else (None, 0, 0, 0)
        res, pact, plo, phi, oq = post if post is not None else (None, 0, 0.0, 0.0, None)
        oq = _quantizer_args(oq) if oq is not None else (None, 0, 0, 0)
        y, ib, iib, ob, oib = _conv2d_block_op(
            _as_f32(x), _as_f32(w), None if qin is not None else _bias_dev(bA, dev), bW_, _bias_dev(bR, dev), tab,
            int(E), int(M), int(flags), [int(s) for s in stride], [int(p) for p in padding],
            [int(d) for d in dilation], int(groups), iq[0].to(dev) if iq[0] is not None else None, iq[1], iq[2],
            iq[3], res, int(pact), float(plo), float(phi), oq[0].to(dev) if oq[0] is not None else None, oq[1],
            oq[2], oq[3], *(epilogue or ()))
        ib._fp8a_i32 = iib
        ob._fp8a_i32 = oib
        _prof_end(ev, y.shape[0] * y.shape[2] * y.shape[3] * w.shape[0] * w.shape[1] * w.shape[2] * w.shape[3])
        return y, (ib if qin is not None else None), (ob if oq[0] is not None else None)
    y = _conv2d_op(_as_f32(x), _as_f32(w), _bias_dev(bA, dev), bW_, _bias_dev(bR, dev), tab,
                   int(E), int(M), int(flags), [int(s) for s in stride], [int(p) for p in padding],
                   [int(d) for d in dilation], int(groups), *(epilogue or ()))
    _prof_end(ev, y.shape[0] * y.shape[2] * y.shape[3] * w.shape[0] * w.shape[1] * w.shape[2] * w.shape[3])
    return y


def bn_act_epilogue(running_mean, running_var, gamma, beta, eps, activation=None):
    """Epilogue parameters for approx_conv2d: eval-mode F.batch_norm as one scale/shift per
    channel (scale = gamma / sqrt(var + eps), shift = beta - mean * scale, the transform ATen's
    eval batch norm applies) and ReLU / ReLU6 / Hardtanh as a clamp.  Returns None when the
    activation is not a clamp (the caller then runs it unfused)."""
    if activation is None:
        act, lo, hi = 0, 0.0, 0.0
    elif type(activation) is nn.ReLU:
        act, lo, hi = 1, 0.0, float("inf")
    elif type(activation) is nn.ReLU6:
        act, lo, hi = 1, 0.0, 6.0
    elif type(activation) is nn.Hardtanh:
        act, lo, hi = 1, float(activation.min_val), float(activation.max_val)
    else:
        return None
    with torch.no_grad():
        invstd = 1.0 / torch.sqrt(running_var.float() + eps)
        scale = invstd * gamma.float() if gamma is not None else invstd
        shift = -running_mean.float() * scale
        if beta is not None:
            shift = shift + beta.float()
        return torch.stack((scale, shift), dim=1).contiguous(), act, lo, hi


# ----------------------------------------------------------------------------------- FP8 fake quant
def fp8_fake_quantize(x, maxval, n_bits, mantissa_bits, sign_bits=1, per_row=False):
    """quantize_to_fp8_ste_MM forward (fp8_quantizer.py:97-173): returns (values, float bias).

    The bias has the reference's shape: [1] per tensor, [C, 1, ..., 1] per channel."""
    L = _lib.load()
    x = _as_f32(x).contiguous()
    mx = _as_f32(maxval).reshape(-1).contiguous()
    if mx.device != x.device:
        mx = mx.to(x.device)
    rows = mx.numel() if per_row else 1
    out = torch.empty_like(x)
    bias = torch.empty(rows, dtype=torch.float32, device=x.device)
    ibias = torch.empty(rows, dtype=torch.int32, device=x.device)
    rc = L.fp8a_fp8_quantize(_lib.dev_ptr(x), rows, x.numel() // rows, _lib.dev_ptr(mx), int(per_row), int(n_bits),
                             int(mantissa_bits), int(sign_bits), _lib.dev_ptr(out), _lib.dev_ptr(bias),
                             _lib.dev_ptr(ibias), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_fp8_quantize")
    if per_row and rows > 1:
        bias = bias.view([-1] + [1] * (x.dim() - 1))
    # the same bias as int32, written by the same kernel: the approx ops take it as is (_bias_dev)
    bias._fp8a_i32 = ibias
    return out, bias


# ----------------------------------------------------------------------------------- qamaa
def _res_quant_params(res_quantizer):
    """(maxval device tensor, n_bits, mantissa bits, sign bits) of a res QuantizationManager /
    FPQuantizer, as approx_multiply reads them (approx_calculation.py:790-794)."""
    q = getattr(res_quantizer, "quantizer", res_quantizer)
    mb = q.mantissa_bits
    mb = int(torch.clamp(torch.round(torch.as_tensor(mb, dtype=torch.float32)), 1, q.n_bits - q.sign_bits).item()) \
        if isinstance(mb, torch.Tensor) else int(mb)
    return q.maxval, int(q.n_bits), mb, int(q.sign_bits)


def qamaa_matmul(A, B, maxval, n_bits, mantissa_bits, sign_bits=1):
    """quantize_after_mult_and_add: fq(sum_k fq(A[m,k] * B[k,n])) on the GPU."""
    if A.dim() != 2 or B.dim() != 2 or A.shape[1] != B.shape[0]:
        raise AssertionError(f"qamaa_matmul: shape mismatch {tuple(A.shape)} @ {tuple(B.shape)}")
    L = _lib.load()
    A, B = _as_f32(A), _as_f32(B)
    if A.stride(1) != 1:
        A = A.contiguous()
    if B.stride(0) != 1 and B.stride(1) != 1:
        B = B.contiguous()
    mx = _as_f32(maxval).reshape(-1).to(A.device).contiguous()
    C = torch.empty((A.shape[0], B.shape[1]), dtype=torch.float32, device=A.device)
    ev = _prof_start()
    rc = L.fp8a_matmul_qamaa(_lib.dev_ptr(A), A.stride(0), _lib.dev_ptr(B), B.stride(0), B.stride(1),
                             _lib.dev_ptr(C), A.shape[0], B.shape[1], A.shape[1], _lib.dev_ptr(mx), int(n_bits),
                             int(mantissa_bits), int(sign_bits), _lib.stream_ptr(A.device))
    _lib.check(rc, "fp8a_matmul_qamaa")
    _prof_end(ev, A.shape[0] * A.shape[1] * B.shape[1])
    return C


def qamaa_conv2d(x, w, maxval, n_bits, mantissa_bits, sign_bits=1, stride=(1, 1), padding=(0, 0),
                 dilation=(1, 1), groups=1):
    """Convolution form of qamaa (groups with > 1 output channel)."""
    L = _lib.load()
    x = _as_f32(x).contiguous()
    w = _as_f32(w).contiguous()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    mx = _as_f32(maxval).reshape(-1).to(x.device).contiguous()
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    rc = L.fp8a_conv2d_qamaa(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, kh, kw,
                             stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1], groups,
                             _lib.dev_ptr(mx), int(n_bits), int(mantissa_bits), int(sign_bits),
                             _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_conv2d_qamaa")
    return y


# ------------------------------------------------------------------- the exact product (dense)
def dense_format(mant_width):
    """fp8a_dense operand format for values on a grid with ``mant_width`` mantissa bits.  Default
    bf16 (every FP8 / E3M4 / E2M5 grid value is exact in bf16 at any exponent; measured exact
    accumulation); FP8A_DENSE_FMT=fp8 selects the block-scaled OCP fp8 form -- e4m3
    for 3 mantissa bits, e5m2 for fewer, None (the fp32 contraction) for wider mantissas."""
    if os.environ.get("FP8A_DENSE_FMT", "bf16") != "fp8":
        return _lib.DENSE_BF16 if 0 < mant_width <= 7 else None
    if mant_width == 3:
        return _lib.DENSE_E4M3
    if 0 < mant_width <= 2:
        return _lib.DENSE_E5M2
    return None


@torch.library.custom_op("fp8approx::dense_matmul", mutates_args=())
def _dense_matmul_op(A: torch.Tensor, B: torch.Tensor, fmt: int) -> torch.Tensor:
    L = _lib.load()
    dev = A.device
    Mr, K = A.shape
    N = B.shape[1]
    C = torch.empty((Mr, N), dtype=torch.float32, device=dev)
    ws = _workspace(dev, L.fp8a_dense_matmul_workspace_size(Mr, N, K))
    rc = L.fp8a_dense_matmul(_lib.dev_ptr(A), A.stride(0), A.stride(1), _lib.dev_ptr(B), B.stride(0), B.stride(1),
                             _lib.dev_ptr(C), N, Mr, N, K, int(fmt), _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(dev))
    _lib.check(rc, "fp8a_dense_matmul")
    return C


@_dense_matmul_op.register_fake
def _(A, B, fmt):
    return A.new_empty((A.shape[0], B.shape[1]), dtype=torch.float32)


def dense_matmul(A, B, fmt):
    """A [M, K] @ B [K, N] (fp32 values on an FP8 grid, any strides) on the matrix core: the
    reference's exact branch ``x @ y`` (approx_calculation.py:797, 811), equal to the fp32 product
    up to summation order (off-grid values: their units in fp32).  fmt: dense_format() -- the bf16
    form (dn_gemm_bf16, v_mfma_f32_16x16x32_bf16) by default, the block-scaled fp8 form
    (v_mfma_scale_f32_16x16x128_f8f6f4) with FP8A_DENSE_FMT=fp8."""
    if A.dim() != 2 or B.dim() != 2 or A.shape[1] != B.shape[0]:
        raise AssertionError(f"dense_matmul: shape mismatch {tuple(A.shape)} @ {tuple(B.shape)}")
    A, B = _as_f32(A), _as_f32(B)
    ev = _prof_start()
    C = _dense_matmul_op(A, B, int(fmt))
    _prof_end(ev, A.shape[0] * A.shape[1] * B.shape[1], 4 * (A.numel() + B.numel() + C.numel()))
    return C


@torch.library.custom_op("fp8approx::dense_conv2d", mutates_args=())
def _dense_conv2d_op(x: torch.Tensor, w: torch.Tensor, fmt: int, stride: list[int], padding: list[int],
                     dilation: list[int]) -> torch.Tensor:
    L = _lib.load()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    geo = (Bn, Cin, H, W, Cout, kh, kw, stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1])
    ws = _workspace(x.device, L.fp8a_dense_conv2d_workspace_size(*geo))
    rc = L.fp8a_dense_conv2d(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), *geo, int(fmt), _lib.dev_ptr(ws),
                             ws.numel(), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_dense_conv2d")
    return y


@_dense_conv2d_op.register_fake
def _(x, w, fmt, stride, padding, dilation):
    Bn, _, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    return x.new_empty((Bn, Cout, Ho, Wo), dtype=torch.float32)


def dense_conv2d(x, w, fmt, stride=(1, 1), padding=(0, 0), dilation=(1, 1)):
    """Exact-product convolution (groups = 1) on the matrix core (the bf16 form by default, the
    block-scaled fp8 form with FP8A_DENSE_FMT=fp8; see dense_matmul): the reference's im2col +
    ``x @ y`` (approx_calculation.py:811) without the im2col image."""
    if x.dim() != 4 or w.dim() != 4 or x.shape[1] != w.shape[1]:
        raise AssertionError(f"dense_conv2d: shape mismatch {tuple(x.shape)} * {tuple(w.shape)}")
    x = _as_f32(x).contiguous()
    w = _as_f32(w).contiguous()
    ev = _prof_start()
    y = _dense_conv2d_op(x, w, int(fmt), [int(v) for v in stride], [int(v) for v in padding],
                         [int(v) for v in dilation])
    _prof_end(ev, y.shape[0] * y.shape[2] * y.shape[3] * w.shape[0] * w.shape[1] * w.shape[2] * w.shape[3],
              4 * (x.numel() + w.numel() + y.numel()))
    return y


@torch.library.custom_op("fp8approx::grouped_conv2d", mutates_args=())
def _grouped_conv2d_op(x: torch.Tensor, w: torch.Tensor, groups: int, stride: list[int], padding: list[int],
                       dilation: list[int]) -> torch.Tensor:
    L = _lib.load()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    rc = L.fp8a_grouped_conv2d(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), Bn, Cin, H, W, Cout, int(groups),
                               kh, kw, stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1],
                               _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_grouped_conv2d")
    return y


@_grouped_conv2d_op.register_fake
def _(x, w, groups, stride, padding, dilation):
    Bn, _, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    return x.new_empty((Bn, Cout, Ho, Wo), dtype=torch.float32)


def grouped_conv2d(x, w, groups, stride=(1, 1), padding=(0, 0), dilation=(1, 1)):
    """Exact-product grouped / depthwise convolution on the HIP kernel fp8a_grouped_conv2d: the
    reference's per-group im2col + ``x @ w^T`` (QCustomConv2dTorch, approx_calculation.py:686-711;
    the exact branch's ``x @ y[:, i]``, :797) -- fp32 FMAs in im2col k order, any fp32 input."""
    if x.dim() != 4 or w.dim() != 4 or x.shape[1] != w.shape[1] * groups or w.shape[0] % groups:
        raise AssertionError(f"grouped_conv2d: shape mismatch {tuple(x.shape)} * {tuple(w.shape)} / {groups}")
    x = _as_f32(x).contiguous()
    w = _as_f32(w).contiguous()
    ev = _prof_start()
    y = _grouped_conv2d_op(x, w, int(groups), [int(v) for v in stride], [int(v) for v in padding],
                           [int(v) for v in dilation])
    _prof_end(ev, y.numel() * w.shape[1] * w.shape[2] * w.shape[3], 4 * (x.numel() + w.numel() + y.numel()))
    return y


def dense_conv2d_fused(x, w, groups=1, stride=(1, 1), padding=(0, 0), dilation=(1, 1), fmt=None, qin=None, rq=None,
                       bn=None, oq=None, wq=None):
    """A config-1 layer in one launch family (fp8a_dense_conv2d_fused): y = oq(clamp(bn(rq(conv(qin(x), wq(w)))))).
    qin / rq / oq: (maxval, n_bits, mantissa bits, sign bits) of a per-tensor FP8 quantizer or None;
    wq: the same for the weight quantizer, per tensor or per output channel (maxval [Cout]); bn:
    (scale_shift [C][2], act, lo, hi) from bn_act_epilogue or None.  Returns (y, biases): each
    given quantizer's float bias tensor (its custom_bias: [1], or [Cout, 1, 1, 1] for a per-channel
    wq, as fp8_fake_quantize returns it), keyed "qin" / "rq" / "oq" / "wq"."""
    if x.dim() != 4 or w.dim() != 4 or x.shape[1] != w.shape[1] * groups or w.shape[0] % groups:
        raise AssertionError(f"dense_conv2d_fused: shape mismatch {tuple(x.shape)} * {tuple(w.shape)} / {groups}")
    L = _lib.load()
    x = _as_f32(x).contiguous()
    w = _as_f32(w).contiguous()
    Bn, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    y = torch.empty((Bn, Cout, Ho, Wo), dtype=torch.float32, device=x.device)
    keep, biases, qargs = [], {}, []
    for name, q in (("wq", wq), ("qin", qin), ("rq", rq), ("oq", oq)):
        if q is None:
            qargs += [None, 0, 0, 0, None, None] if name != "wq" else [None, 0, 0, 0, 0, None, None]
            continue
        mx = _as_f32(q[0]).reshape(-1).to(x.device).contiguous()
        rows = mx.numel()
        if name == "wq" and rows not in (1, Cout):
            raise AssertionError(f"dense_conv2d_fused: weight quantizer with {rows} maxvals for {Cout} channels")
        if name != "wq" and rows != 1:
            raise AssertionError(f"dense_conv2d_fused: {name} must be a per-tensor quantizer")
        b = torch.empty(rows, dtype=torch.float32, device=x.device)
        ib = torch.empty(rows, dtype=torch.int32, device=x.device)
        keep.append(mx)
        head = [_lib.dev_ptr(mx)] + ([int(rows > 1)] if name == "wq" else [])
        qargs += head + [int(q[1]), int(q[2]), int(q[3]), _lib.dev_ptr(b), _lib.dev_ptr(ib)]
        if rows > 1:
            b = b.view(-1, 1, 1, 1)
        b._fp8a_i32 = ib
        biases[name] = b
    ep, act, lo, hi = (None, 0, 0.0, 0.0) if bn is None else bn
    if ep is not None:
        ep = _as_f32(ep).to(x.device).contiguous()
    geo = (Bn, Cin, H, W, Cout, kh, kw, stride[0], stride[1], padding[0], padding[1], dilation[0], dilation[1])
    ws = _workspace(x.device, L.fp8a_dense_conv2d_workspace_size(*geo) if groups == 1 else 16)
    fmt = dense_format(3) if fmt is None else fmt
    ev = _prof_start()
    rc = L.fp8a_dense_conv2d_fused(_lib.dev_ptr(x), _lib.dev_ptr(w), _lib.dev_ptr(y), *geo, int(groups), int(fmt),
                                   *qargs[:19], _lib.dev_ptr(ep) if ep is not None else None, int(act), float(lo),
                                   float(hi), *qargs[19:], _lib.dev_ptr(ws), ws.numel(), _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_dense_conv2d_fused")
    _prof_end(ev, y.numel() * w.shape[1] * kh * kw, 4 * (x.numel() + w.numel() + y.numel()))
    return y, biases


# ----------------------------------------------------------------------------------- max pool
@torch.library.custom_op("fp8approx::max_pool2d", mutates_args=())
def _max_pool2d_op(x: torch.Tensor, kernel: list[int], stride: list[int], padding: list[int]) -> torch.Tensor:
    L = _lib.load()
    x = x.contiguous()
    Bn, C, H, W = x.shape
    Ho = (H + 2 * padding[0] - kernel[0]) // stride[0] + 1
    Wo = (W + 2 * padding[1] - kernel[1]) // stride[1] + 1
    y = torch.empty((Bn, C, Ho, Wo), dtype=x.dtype, device=x.device)
    rc = L.fp8a_max_pool2d(_lib.dev_ptr(x), _lib.dev_ptr(y), Bn, C, H, W, kernel[0], kernel[1], stride[0], stride[1],
                           padding[0], padding[1], _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_max_pool2d")
    return y


@_max_pool2d_op.register_fake
def _(x, kernel, stride, padding):
    Bn, C, H, W = x.shape
    return x.new_empty((Bn, C, (H + 2 * padding[0] - kernel[0]) // stride[0] + 1,
                        (W + 2 * padding[1] - kernel[1]) // stride[1] + 1))


class MaxPool2d(nn.Module):
    """nn.MaxPool2d (dilation 1, floor mode) on the HIP kernel fp8a_max_pool2d; same values
    (max is exact, NaN propagates).  ``from_module`` keeps other configurations on torch."""

    def __init__(self, kernel_size, stride, padding):
        super().__init__()
        pair = lambda v: [int(v), int(v)] if isinstance(v, int) else [int(t) for t in v]  # noqa: E731
        self.kernel_size, self.stride, self.padding = pair(kernel_size), pair(stride), pair(padding)

    @staticmethod
    def from_module(m):
        if (type(m) is nn.MaxPool2d and m.dilation in (1, (1, 1)) and not m.ceil_mode and not m.return_indices
                and m.stride is not None):
            mp = MaxPool2d(m.kernel_size, m.stride, m.padding)
            if all(2 * p <= k for p, k in zip(mp.padding, mp.kernel_size)):
                return mp
        return m

    def forward(self, x):
        if x.dtype != torch.float32 or x.dim() != 4 or not x.is_cuda:
            return nn.functional.max_pool2d(x, self.kernel_size, self.stride, self.padding)
        return _max_pool2d_op(x, self.kernel_size, self.stride, self.padding)

    def extra_repr(self):
        return f"kernel_size={self.kernel_size}, stride={self.stride}, padding={self.padding} (HIP)"


# ----------------------------------------------------------------------------------- avg pool
@torch.library.custom_op("fp8approx::avg_pool2d_plane", mutates_args=())
def _avg_pool2d_plane_op(x: torch.Tensor, kernel: list[int], stride: list[int]) -> torch.Tensor:
    L = _lib.load()
    x = x.contiguous()
    Bn, C, H, W = x.shape
    y = torch.empty((Bn, C, 1, 1), dtype=x.dtype, device=x.device)
    rc = L.fp8a_avg_pool2d_plane(_lib.dev_ptr(x), _lib.dev_ptr(y), Bn, C, H, W, kernel[0], kernel[1], stride[0],
                                 stride[1], _lib.stream_ptr(x.device))
    _lib.check(rc, "fp8a_avg_pool2d_plane")
    return y


@_avg_pool2d_plane_op.register_fake
def _(x, kernel, stride):
    return x.new_empty((x.shape[0], x.shape[1], 1, 1))


class AvgPool2d(nn.AvgPool2d):
    """nn.AvgPool2d (padding 0, floor mode, no divisor override) whose output is one value per
    plane -- the MobileNetV2 head's AvgPool2d(input_size // 32) -- on the HIP kernel
    fp8a_avg_pool2d_plane: the window summed in row-major order in fp32 and divided by kh kw, as
    ATen's avg_pool2d does (the same bits).  Other inputs / geometries run torch's pooling; still an
    nn.AvgPool2d, so quantize_sequential wraps it like the original (model_wrap.py)."""

    def __init__(self, kernel_size, stride=None):
        super().__init__(kernel_size, stride)

    def forward(self, x):
        pair = lambda v: [int(v), int(v)] if isinstance(v, int) else [int(t) for t in v]  # noqa: E731
        k, s = pair(self.kernel_size), pair(self.stride)
        if (x.dtype == torch.float32 and x.dim() == 4 and x.is_cuda and k[0] <= x.shape[2] < k[0] + s[0]
                and k[1] <= x.shape[3] < k[1] + s[1] and x.shape[2] * x.shape[3] <= 4096):
            return _avg_pool2d_plane_op(x, k, s)
        return super().forward(x)
