"""The superseded integer-adder approximate multiplier, v5 (opt-in), on the GPU.

Mirrors approx/approx_matmul_whole_v5.py of revollllt/FP8_quantization @ 2024-11-08: the
product of two FP8 values is approximated by ADDING their (expo << M | mant) integer codes,
subtracting bias << M and adding a compensation table entry (approx_mult_new, v5:155-183);
sim_hw_add_OFUF wraps the sum like an (E+M)-bit hardware adder, with_OF_opt / with_UF_opt
repair overflow / underflow.  v9 -- which the reference's operators call -- accepts these
switches and ignores them; this module is where they act.

Differences from the reference, on purpose:
  * v5's ``with_OF_opt`` line builds its replacement value with ``device=A.device`` where ``A``
    is not a local name, so outside v5's own ``__main__`` it raises NameError; here the branch
    computes the value it evidently means (overflow -> max_norm_int).  The golden vectors
    (tests/golden/g7_v5.npz) pin that value: the generator gave the module the global it reads.
  * the engine generalises v5's single ``custom_bias`` to per-operand biases (bA, bB, bR):
    the code sum subtracts (bA + bB - bR) << M; with bA = bB = bR it is v5 exactly.  That is
    what the operator-level opt-in (custom_approx_params["approx_version"] = 5) uses.
"""
import torch

from . import _lib
from .approx_ops import approx_conv2d, approx_matmul, make_flags_v5
from .error_tables import get_comp_table_NN_v5

__all__ = ["custom_matmul_vectorize", "get_comp_table_NN", "approx_matmul_v5", "approx_conv2d_v5", "param_prepare"]


def param_prepare(expo_width, mant_width, custom_bias=None, debug_mode=False):
    """v5's parameter dictionary (approx_matmul_whole_v5.py:204-241)."""
    fp_bias = custom_bias if custom_bias is not None else int(2 ** (expo_width - 1) - 1)
    max_expo = int(2 ** expo_width - 1)
    d = dict(fp_bias=fp_bias, bias_double=int(2 * fp_bias), max_norm=(2 ** (max_expo - fp_bias)) * (2 - 2 ** -mant_width),
             min_norm=2 ** (1 - fp_bias), min_subnorm=(2 ** (1 - fp_bias)) * 2 ** -mant_width, max_expo=max_expo,
             max_mant=int(2 ** mant_width - 1), mant_scale=int(2 ** mant_width),
             max_norm_int=int(2 ** (expo_width + mant_width) - 1), OF_UF_mod=int(2 ** (expo_width + mant_width)))
    if debug_mode:
        for k, v in d.items():
            print(f"{type(v)} : {k} = {v}")
    return d


def get_comp_table_NN(expo_width, mant_width, withComp, dnsmp_factor, device=None):
    """v5's table selection (v5:516-541); the table is returned on the host (it is packed into
    the launch arguments), ``device`` is accepted for signature compatibility."""
    return get_comp_table_NN_v5(expo_width, mant_width, withComp, dnsmp_factor)


def _table(comp_table_NN, mant_width):
    n = 2 ** mant_width
    if comp_table_NN is None:
        return torch.zeros((n, n), dtype=torch.int32)
    return torch.as_tensor(comp_table_NN).to(device="cpu", dtype=torch.int32).contiguous()


def approx_matmul_v5(A, B, E, M, bA, bB, bR, comp_table_NN=None, sim_hw_add_OFUF=False, with_OF_opt=False,
                     with_UF_opt=False):
    """C = sum_k v5 term(A[m, k], B[k, n]) with per-operand biases (bB int or per column)."""
    return approx_matmul(A, B, E, M, bA, bB, bR, _table(comp_table_NN, M),
                         flags=make_flags_v5(sim_hw_add_OFUF, with_OF_opt, with_UF_opt))


def approx_conv2d_v5(x, w, E, M, bA, bW, bR, comp_table_NN=None, sim_hw_add_OFUF=False, with_OF_opt=False,
                     with_UF_opt=False, **conv):
    return approx_conv2d(x, w, E, M, bA, bW, bR, _table(comp_table_NN, M),
                         flags=make_flags_v5(sim_hw_add_OFUF, with_OF_opt, with_UF_opt), **conv)


def custom_matmul_vectorize(A, B, expo_width, mant_width, custom_bias, comp_table_NN, sim_hw_add_OFUF=False,
                            with_OF_opt=False, with_UF_opt=False, golden_clip_OF=False, debug_mode=False,
                            self_check_mode=False):
    """Drop-in for approx_matmul_whole_v5.custom_matmul_vectorize (v5:10-152): one bias for A,
    B and the result (None = 2^(E-1) - 1)."""
    assert A.shape[1] == B.shape[0]
    b = param_prepare(expo_width, mant_width, custom_bias)["fp_bias"]
    out = approx_matmul_v5(A, B, expo_width, mant_width, b, b, b, comp_table_NN, sim_hw_add_OFUF, with_OF_opt,
                           with_UF_opt)
    if self_check_mode:
        from .approx_ops import quant_to_fp_any_vectorize_torch
        golden = quant_to_fp_any_vectorize_torch(A.unsqueeze(2) * B.unsqueeze(0), expo_width, mant_width, b,
                                                 clip_OF=golden_clip_OF).sum(dim=1)
        err = (golden - out).abs()
        print("\n====== Self-Checking Mode ======")
        print(f"Max  Error : {err.max()}")
        print(f"Mean Error : {err.mean()}")
        print(f"RMSE       : {torch.sqrt(torch.mean(err ** 2))}")
    return out
