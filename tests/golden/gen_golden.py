#!/usr/bin/env python
"""Golden-vector generator for the approx_v9 hot path (TEST INFRASTRUCTURE ONLY).

Runs ONLY in the build container, where the reference checkout is mounted read-only at
/root/reference.  It imports the reference UNMODIFIED through a small import shim (SURVEY.md
§8(c)): module-level ``device='cuda'`` tensors are redirected to the CPU, and the
un-installed ``cupy`` / ``timm`` imports are satisfied by empty stub modules.  Nothing here is
shipped; the GPU box only sees the ``.npz`` fixtures this script writes next to itself.

Fixture groups:
  g1_decompose.npz  DEC / Q_R known-answer table      (approx_matmul_whole_v9.py:189-362)
  g2_matmul.npz     custom_matmul_vectorize, scalar biases, flag matrix, sums + per-term
                    values                            (approx_matmul_whole_v9.py:10-169)
  g3_debug.npz      the captured MobileNetV2 layer in debug_params/*.csv through the
                    per-column loop of approx_multiply (approx_calculation.py:749-814)
  g4_tensorbias.npz single-column (tensor-bias) calls, quirk F5 (approx_calculation.py:800-809)
  g5_operator.npz   QCustomBNConv2dTorch / QCustomLinearTorch through estimate->fix->approx
                    (quantized_folded_bn.py:30-83, hijacker.py:77-115)
  g6_qamaa.npz      the quantize_after_mult_and_add branch of approx_multiply
                    (approx_calculation.py:787-795)
  g7_v5.npz         the superseded integer-adder model with live sim_hw_add_OFUF /
                    with_OF_opt / with_UF_opt semantics (approx_matmul_whole_v5.py:10-183,
                    tables :362-550); v5's with_OF_opt line names a global `A` that only the
                    module's own __main__ defines, so the generator sets one (a CPU tensor, used
                    for its .device only) to let that branch run
  g8_mbv2.npz       model level: the reference's QuantizedMobileNetV2
                    (models/mobilenet_v2_quantized_approx.py) over its float MobileNetV2
                    (width 0.25, 32x32, 10 classes, random weights and BN statistics) through
                    estimate -> fix -> approx: the initial state, every layer's biases, logits,
                    and per approx layer of the fixed-range forward its run_forward operands /
                    product and its own input / output (teacher-forced layer tests)

Usage:  python tests/golden/gen_golden.py      (about a minute on 8 cores)
"""
import io
import contextlib
import json
import os
import random
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- import shim
def _install_shim():
    orig_tensor, orig_zeros = torch.tensor, torch.zeros

    def _cpu(kw):
        d = kw.get("device")
        if d is not None and str(d).startswith("cuda"):
            kw["device"] = "cpu"
        return kw

    torch.tensor = lambda *a, **kw: orig_tensor(*a, **_cpu(kw))
    torch.zeros = lambda *a, **kw: orig_zeros(*a, **_cpu(kw))
    sys.modules.setdefault("cupy", types.ModuleType("cupy"))
    mods = ["timm", "timm.models", "timm.models.layers",
            "timm.models.layers.activations", "timm.models.layers.activations_me"]
    for m in mods:
        sys.modules.setdefault(m, types.ModuleType(m))
    for c in ("Swish", "HardSwish", "HardSigmoid"):
        setattr(sys.modules["timm.models.layers.activations"], c, type(c, (nn.Module,), {}))
    for c in ("SwishMe", "HardSwishMe", "HardSigmoidMe"):
        setattr(sys.modules["timm.models.layers.activations_me"], c, type(c, (nn.Module,), {}))
    sys.path.insert(0, REF)


_install_shim()
import approx.approx_matmul_whole_v9 as v9  # noqa: E402  (reference, unmodified)
import approx.approx_calculation as ac  # noqa: E402
import approx.approx_matmul_whole_v5 as v5  # noqa: E402  (reference, unmodified)
from quantization.quantizers.fp8_quantizer import FPQuantizer  # noqa: E402
from quantization.range_estimators import RangeEstimators  # noqa: E402

FORMATS = [(4, 3), (3, 4), (2, 5), (5, 2)]


def table(E, M, with_comp=False, dnsmp_factor=3, withComp=None):
    """Error table as the operator would pick it; E5M2 (unsupported by the reference,
    SURVEY F3) gets an all-zero table so its arithmetic can still be pinned.  (Also stands in
    for the reference's get_error_table_NN signature, withComp= keyword included.)"""
    if withComp is not None:
        with_comp = withComp
    if (E, M) == (5, 2):
        return torch.zeros((4, 4), dtype=torch.int32)
    return v9.get_error_table_NN(E, M, withComp=with_comp, dnsmp_factor=dnsmp_factor)


TABLE_VARIANTS = {
    (4, 3): [("comp", True, 3), ("nocomp", False, 3)],
    (3, 4): [("comp3", True, 3), ("comp4", True, 4), ("nocomp", False, 3)],
    (2, 5): [("comp3", True, 3), ("comp4", True, 4), ("comp5", True, 5), ("nocomp", False, 3)],
    (5, 2): [("zero", True, 3)],
}


# ----------------------------------------------------------------------------- G1
def grid_values(E, M, b, extra_expo=3):
    vals = []
    for expo in range(0, 2 ** E + extra_expo):
        for mant in range(2 ** M):
            if expo == 0:
                vals.append(2.0 ** (1 - b) * mant / 2 ** M)
            else:
                vals.append(2.0 ** (expo - b) * (1 + mant / 2 ** M))
    v = np.array(vals, dtype=np.float64)
    return np.concatenate([v, -v])


def edge_values(E, M, b, rng):
    min_norm = 2.0 ** (1 - b)
    min_sub = min_norm * 2.0 ** -M
    max_norm = 2.0 ** (2 ** E - 1 - b) * (2 - 2.0 ** -M)
    f32 = np.float32
    e = [0.0, min_sub / 2, min_sub * 0.5000001, min_sub * 0.4999999, min_sub * 1.5, min_sub * 2.5,
         min_norm * (1 - 2.0 ** -(M + 2)), min_norm * (1 - 2.0 ** -(M + 1)),
         float(np.nextafter(f32(min_norm), f32(0))), min_norm,
         max_norm, max_norm * 1.01, max_norm * 4, 1e30, 1e-30, 1e-40, 3e-39]
    for ex in range(-6, 6):
        base = 2.0 ** ex
        e += [base * (2 - 2.0 ** -M - 2.0 ** -(M + 2)), base * (2 - 2.0 ** -(M + 1)),
              base * (2 - 2.0 ** -(M + 1)) * (1 + 1e-6), base * (1 + 2.0 ** -(M + 1)),
              base * (1 + 3 * 2.0 ** -(M + 1))]
    rnd = rng.standard_normal(300) * 2.0 ** rng.integers(-24, 10, 300)
    v = np.concatenate([np.array(e), rnd])
    return np.concatenate([v, -v])


def gen_g1():
    rng = np.random.default_rng(1234)
    out, meta = {}, []
    for (E, M) in FORMATS:
        for b in sorted({2 ** (E - 1) - 1, 3, 5, 9, 14, 19}):
            x = np.concatenate([grid_values(E, M, b), edge_values(E, M, b, rng)]).astype(np.float32)
            x[len(x) // 2] = -0.0
            xt = torch.from_numpy(x.copy())
            key = f"E{E}M{M}_b{b}"
            out[key + "_x"] = x
            for tb in (False, True):
                bias = torch.tensor([b], dtype=torch.int32) if tb else b
                for clip in (False, True):
                    pd = v9.param_prepare(E, M, custom_bias=bias)
                    expo, mant = v9.float_to_fpany_absint_torch(pd, xt.clone(), clip_OF=clip)
                    q = v9.quant_to_fp_any_vectorize_torch(xt.clone(), E, M, custom_bias=bias,
                                                           clip_OF=clip)
                    sfx = f"_tb{int(tb)}_c{int(clip)}"
                    out[key + sfx + "_expo"] = expo.numpy().astype(np.int32)
                    out[key + sfx + "_mant"] = mant.numpy().astype(np.int32)
                    out[key + sfx + "_q"] = q.numpy().astype(np.float32)
            meta.append(dict(key=key, E=E, M=M, b=b))
    np.savez_compressed(os.path.join(HERE, "g1_decompose.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G2
def random_grid_tensor(E, M, bias, rows, cols, seed):
    """Same draw as the reference self-check harness (approx_matmul_whole_v9.py:794-804):
    numpy picks a code of the value space, python's random picks the sign."""
    np.random.seed(seed)
    random.seed(seed)
    space = v9.show_value_space(E, M, bias, show_style=0).numpy()
    return torch.tensor([[np.random.choice(space) * random.choice([-1, 1]) for _ in range(cols)]
                         for _ in range(rows)], dtype=torch.float32)


G2_BIASES = {(3, 4): (3, 5, 5), (4, 3): (7, 9, 8), (2, 5): (1, 2, 2), (5, 2): (15, 17, 16)}


def cmv(A, B, E, M, bA, bB, bR, tab, approx, s2n, qbma, gclip):
    with contextlib.redirect_stdout(io.StringIO()):
        return v9.custom_matmul_vectorize(
            A, B, E, M, bA, bB, bR, tab, with_approx=approx, with_s2nn2s_opt=s2n,
            golden_clip_OF=gclip, quant_btw_mult_accu=qbma)


def gen_g2():
    out, meta = {}, []
    for (E, M), (bA, bB, bR) in G2_BIASES.items():
        n = 256 if (E, M) == (3, 4) else 128
        A = random_grid_tensor(E, M, bA, n, n, seed=5)
        B = random_grid_tensor(E, M, bB, n, n, seed=5 if (E, M) == (3, 4) else 6)
        fk = f"E{E}M{M}"
        out[fk + "_A"] = A.numpy()
        out[fk + "_B"] = B.numpy()
        Ac, Bc = A[:64], B[:, :64]
        At, Bt = A[:8, :64], B[:64, :8]
        for (tname, wc, dn) in TABLE_VARIANTS[(E, M)]:
            tab = table(E, M, wc, dn)
            for approx in (True, False):
                if not approx and tname != TABLE_VARIANTS[(E, M)][0][0]:
                    continue  # table is irrelevant without approx
                for s2n in (True, False):
                    for qbma in (True, False):
                        for gclip in (False, True):
                            key = f"{fk}_{tname}_a{int(approx)}_s{int(s2n)}_q{int(qbma)}_g{int(gclip)}"
                            C = cmv(Ac, Bc, E, M, bA, bB, bR, tab, approx, s2n, qbma, gclip)
                            out[key + "_C"] = C.numpy()
                            terms = torch.stack([cmv(At[:, k:k + 1], Bt[k:k + 1, :], E, M, bA, bB, bR,
                                                     tab, approx, s2n, qbma, gclip)
                                                 for k in range(At.shape[1])], dim=1)
                            out[key + "_T"] = terms.numpy()
                            meta.append(dict(key=key, fmt=fk, E=E, M=M, bA=bA, bB=bB, bR=bR,
                                             table=tname, with_comp=wc, dnsmp=dn, approx=approx,
                                             s2n=s2n, qbma=qbma, gclip=gclip))
        for (tname, wc, dn) in TABLE_VARIANTS[(E, M)]:
            out[f"{fk}_table_{tname}"] = table(E, M, wc, dn).numpy().astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "g2_matmul.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G3
class _FakeOp:
    """Minimal stand-in carrying the attributes approx_multiply reads."""

    def __init__(self, params, approx_flag=True):
        self.custom_approx_params = params
        self.approx_flag = approx_flag
        self.quantize_after_mult_and_add = False


def approx_params(E, M, dnsmp, with_comp, approx, s2n, qbma, gclip=False):
    return dict(expo_width=E, mant_width=M, dnsmp_factor=dnsmp, withComp=with_comp,
                with_approx=approx, with_s2nn2s_opt=s2n, sim_hw_add_OFUF=False,
                with_OF_opt=False, with_UF_opt=False, golden_clip_OF=gclip,
                quant_btw_mult_accu=qbma, debug_mode=False, self_check_mode=False)


def gen_g3():
    A = np.loadtxt(os.path.join(REF, "debug_params/act.csv"), delimiter=",", dtype=np.float32)
    B = np.loadtxt(os.path.join(REF, "debug_params/weight.csv"), delimiter=",", dtype=np.float32)
    bA = np.loadtxt(os.path.join(REF, "debug_params/act_bias.csv"), delimiter=",", dtype=np.float32).reshape(1)
    bB = np.loadtxt(os.path.join(REF, "debug_params/weight_bias.csv"), delimiter=",", dtype=np.float32).reshape(-1)
    bR = np.array([5.0], dtype=np.float32)
    out = dict(A=A, B=B, bA=bA, bB=bB, bR=bR)
    meta = []
    combos = [("comp3", True, 3, True, True, True), ("nocomp", False, 3, True, False, True),
              ("nocomp", False, 3, True, True, False), ("comp4", True, 4, False, False, False),
              ("comp3", True, 3, True, False, True)]
    for (tname, wc, dn, approx, s2n, qbma) in combos:
        op = _FakeOp(approx_params(3, 4, dn, wc, approx, s2n, qbma))
        C = ac.QCustomBNConv2dTorch.approx_multiply(op, torch.from_numpy(A), torch.from_numpy(B),
                                                    torch.from_numpy(bA), torch.from_numpy(bB),
                                                    torch.from_numpy(bR))
        key = f"{tname}_a{int(approx)}_s{int(s2n)}_q{int(qbma)}"
        out[key + "_C"] = C.numpy()
        meta.append(dict(key=key, table=tname, with_comp=wc, dnsmp=dn, approx=approx, s2n=s2n, qbma=qbma))
    np.savez_compressed(os.path.join(HERE, "g3_debug.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G4
def gen_g4():
    out, meta = {}, []
    gen = torch.Generator().manual_seed(77)
    for (E, M), (bA, bB, bR) in G2_BIASES.items():
        if (E, M) == (5, 2):
            continue
        A = random_grid_tensor(E, M, bA, 64, 9, seed=11)
        A[torch.rand(A.shape, generator=gen) < 0.4] = 0.0  # ReLU-like zeros: exercise quirk F5
        Bw = random_grid_tensor(E, M, bB, 9, 1, seed=12)
        fk = f"E{E}M{M}"
        out[fk + "_A"], out[fk + "_B"] = A.numpy(), Bw.numpy()
        for (tname, wc, dn) in TABLE_VARIANTS[(E, M)]:
            for approx in (True, False):
                for s2n in (True, False):
                    for qbma in (True, False):
                        op = _FakeOp(approx_params(E, M, dn, wc, approx, s2n, qbma))
                        xb = torch.tensor([float(bA)])
                        yb = torch.tensor(float(bB))  # 0-dim, as weight_group_fp_bias.squeeze()
                        rb = torch.tensor([float(bR)])
                        C = ac.QCustomBNConv2dTorch.approx_multiply(op, A, Bw, xb, yb, rb)
                        key = f"{fk}_{tname}_a{int(approx)}_s{int(s2n)}_q{int(qbma)}"
                        out[key + "_C"] = C.numpy()
                        terms = torch.stack([
                            ac.QCustomBNConv2dTorch.approx_multiply(op, A[:, k:k + 1], Bw[k:k + 1, :],
                                                                     xb, yb, rb)
                            for k in range(A.shape[1])], dim=1)
                        out[key + "_T"] = terms.numpy()
                        meta.append(dict(key=key, fmt=fk, E=E, M=M, bA=bA, bB=bB, bR=bR, table=tname,
                                         with_comp=wc, dnsmp=dn, approx=approx, s2n=s2n, qbma=qbma))
    np.savez_compressed(os.path.join(HERE, "g4_tensorbias.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G6
class _FakeResQ:
    """The attributes approx_multiply's qamaa branch reads (approx_calculation.py:790-794)."""

    def __init__(self, maxval, M):
        self.quantizer = types.SimpleNamespace(n_bits=8, maxval=torch.tensor([maxval]),
                                               mantissa_bits=torch.tensor([float(M)]), sign_bits=1)


def gen_g6():
    """quantize_after_mult_and_add: per-product FP8 fake quant, sum, fake quant."""
    out, meta = {}, []
    for (E, M), (bA, bB, bR) in G2_BIASES.items():
        if (E, M) == (5, 2):
            continue
        fk = f"E{E}M{M}"
        A = random_grid_tensor(E, M, bA, 48, 96, seed=21)
        B = random_grid_tensor(E, M, bB, 96, 24, seed=22)
        out[fk + "_A"], out[fk + "_B"] = A.numpy(), B.numpy()
        for mx in (0.75, 3.0, 40.0):
            op = _FakeOp(approx_params(E, M, 3, True, True, True, True), approx_flag=False)
            op.quantize_after_mult_and_add = True
            op.res_quantizer = _FakeResQ(mx, M)
            C = ac.QCustomBNConv2dTorch.approx_multiply(op, A, B, torch.tensor([float(bA)]),
                                                        torch.full((24,), float(bB)), torch.tensor([float(bR)]))
            key = f"{fk}_mx{mx}"
            out[key + "_C"] = C.numpy()
            meta.append(dict(key=key, fmt=fk, E=E, M=M, maxval=mx))
    np.savez_compressed(os.path.join(HERE, "g6_qamaa.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G7
# (E5M2 last, so the seeded draws of the other formats are unchanged: v5 has no E5M2 table
# either -- get_comp_table_NN raises for it -- so it runs with the zero table only)
V5_TABLES = {(4, 3): [3], (3, 4): [3, 4], (2, 5): [3, 4, 5], (5, 2): []}
V5_FLAGS = [(False, False, False), (True, False, False), (True, True, False), (True, False, True),
            (True, True, True)]


def v5_operands(E, M, b, rows, cols, rng):
    """Grid codes over the whole exponent range plus out-of-range and off-grid values:
    zeros, subnormals, values above max_norm (clipped by v5's clip_OF=True decode)."""
    expo = rng.integers(0, 2 ** E, size=(rows, cols))
    mant = rng.integers(0, 2 ** M, size=(rows, cols))
    v = np.where(expo == 0, np.ldexp(mant / 2 ** M, 1 - b), np.ldexp(1.0 + mant / 2 ** M, expo - b))
    r = rng.random((rows, cols))
    v = np.where(r < 0.1, 0.0, v)
    big = 2.0 ** (2 ** E - 1 - b) * rng.uniform(2.0, 8.0, size=(rows, cols))
    v = np.where((r >= 0.1) & (r < 0.15), big, v)
    off = np.ldexp(rng.uniform(1.0, 2.0, size=(rows, cols)), rng.integers(-b - 2, 2 ** E - b, size=(rows, cols)))
    v = np.where((r >= 0.15) & (r < 0.25), off, v)
    v = v * rng.choice([-1.0, 1.0], size=(rows, cols))
    return torch.tensor(v, dtype=torch.float32)


def v5_call(A, B, E, M, b, tab, ofuf, of, uf):
    v5.A = torch.zeros(1)  # the global v5's with_OF_opt branch reads (see module docstring)
    with contextlib.redirect_stdout(io.StringIO()):
        return v5.custom_matmul_vectorize(A, B, E, M, custom_bias=b, comp_table_NN=tab, sim_hw_add_OFUF=ofuf,
                                          with_OF_opt=of, with_UF_opt=uf, golden_clip_OF=False)


def gen_g7():
    out, meta = {}, []
    rng = np.random.default_rng(77)
    for (E, M), dns in V5_TABLES.items():
        fk = f"E{E}M{M}"
        tabs = [("zero", torch.zeros((2 ** M, 2 ** M), dtype=torch.int32))]
        for d in dns:
            t = v5.get_comp_table_NN(E, M, True, d, "cpu")
            out[f"{fk}_table_d{d}"] = t.numpy().astype(np.int32)
            tabs.append((f"d{d}", t))
        for b in (None, 2 ** (E - 1) + 2):
            bb = 2 ** (E - 1) - 1 if b is None else b
            A = v5_operands(E, M, bb, 24, 40, rng)
            B = v5_operands(E, M, bb, 40, 16, rng)
            bk = f"{fk}_b{bb}"
            out[bk + "_A"], out[bk + "_B"] = A.numpy(), B.numpy()
            At, Bt = A[:6], B[:, :6]
            for tname, tab in tabs:
                for (ofuf, of, uf) in V5_FLAGS:
                    key = f"{bk}_{tname}_s{int(ofuf)}{int(of)}{int(uf)}"
                    out[key + "_C"] = v5_call(A, B, E, M, b, tab, ofuf, of, uf).numpy()
                    out[key + "_T"] = torch.stack([v5_call(At[:, k:k + 1], Bt[k:k + 1, :], E, M, b, tab, ofuf, of, uf)
                                                   for k in range(At.shape[1])], dim=1).numpy()
                    meta.append(dict(key=key, fmt=fk, E=E, M=M, bias=bb, default_bias=b is None, table=tname,
                                     ofuf=ofuf, of_opt=of, uf_opt=uf))
    np.savez_compressed(os.path.join(HERE, "g7_v5.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G8
def gen_g8():
    # models/__init__.py imports every wrapper, some of which need torchvision (absent here):
    # register the package without running its __init__, then import the two modules unmodified
    if "models" not in sys.modules:
        pkg = types.ModuleType("models")
        pkg.__path__ = [os.path.join(REF, "models")]
        sys.modules["models"] = pkg
    from models.mobilenet_v2 import MobileNetV2 as RefMobileNetV2  # reference, unmodified
    from models.mobilenet_v2_quantized_approx import QuantizedMobileNetV2 as RefQuantizedMobileNetV2
    out, meta = {}, []
    approx_rm = dict(approx_flag=True, quantize_after_mult_and_add=False, res_quantizer_flag=True,
                     original_quantize_res=False)
    # the reference's canonical --no-approx_flag run (scripts/image_net.sh:42-45): the exact product
    # then the res quantizer, through the original_quantize_res branch (quantized_folded_bn.py:40-48;
    # without it the fixed-range forward reads an unassigned `res`)
    exact_rm = dict(approx_rm, approx_flag=False, original_quantize_res=True)
    # mbv2_e4m3: BASELINE config 3's network in E4M3; mbv2_e4m3_noapprox: BASELINE config 1 (E4M3
    # PTQ, --no-approx_flag: the quantizers around the exact product, hijacker.py:88-115);
    # mbv2_e5m2: config 3's format, which the reference's get_error_table_NN rejects (v9:588-590,
    # SURVEY F3) -- the generator gives the reference's operators an all-zero E5M2 table (the
    # engine's opt-in zero_table_ext), everything else is the reference's own code
    cases = [("mbv2_e4m3", (4, 3), False, approx_rm), ("mbv2_e4m3_noapprox", (4, 3), False, exact_rm),
             ("mbv2_e5m2", (5, 2), False, approx_rm)]
    for (name, (E, M), wc, run_method) in cases:
        ac.get_error_table_NN = table if (E, M) == (5, 2) else v9.get_error_table_NN
        torch.manual_seed(88)
        fp = RefMobileNetV2(n_class=10, input_size=32, width_mult=0.25)
        with torch.no_grad():
            for m in fp.modules():
                if isinstance(m, nn.BatchNorm2d):
                    m.weight.uniform_(0.5, 1.5)
                    m.bias.uniform_(-0.2, 0.2)
                    m.running_mean.uniform_(-0.1, 0.1)
                    m.running_var.uniform_(0.5, 2.0)
                elif isinstance(m, nn.Linear):
                    m.weight.normal_(0, 0.1)
                    m.bias.uniform_(-0.1, 0.1)
        qp = qparams_for(E, M, approx_params(E, M, 3, wc, True, True, True), dict(run_method))
        with contextlib.redirect_stdout(io.StringIO()):
            model = RefQuantizedMobileNetV2(fp, input_size=(1, 3, 32, 32), **qp)
        state = {k: v.clone() for k, v in model.state_dict().items()}
        x_cal = torch.randn(4, 3, 32, 32)
        x_ev = torch.randn(3, 3, 32, 32)
        model.eval()
        model.quantized()
        model.estimate_ranges()
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            model(x_cal)
        model.fix_ranges()
        # per approx layer of the fixed-range forward: what run_forward received (the quantized
        # input and weight, the layer's own bias) and returned -- the product the engine replaces --
        # and the layer's own input / output (approx_calculation.py:822-917, 1007-1023;
        # quantized_folded_bn.py:30-83): the engine is teacher-forced on these, layer by layer
        rec, hooks = {}, []
        for lname, mod in model.named_modules():
            if isinstance(mod, (ac.QCustomBNConv2dTorch, ac.QCustomLinearTorch)):
                def run_forward(x, weight, bias, offsets=None, _m=mod, _n=lname, _f=type(mod).run_forward):
                    y = _f(_m, x, weight, bias, offsets)
                    rec[_n + "__x"], rec[_n + "__w"], rec[_n + "__y"] = x.clone(), weight.clone(), y.clone()
                    return y
                mod.run_forward = run_forward

                def io_hook(m, inp, outp, _n=lname):
                    rec[_n + "__in"], rec[_n + "__out"] = inp[0].clone(), outp.clone()
                hooks.append(mod.register_forward_hook(io_hook))
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            logits = model(x_ev)
        for h in hooks:
            h.remove()
        for k, v in rec.items():
            out[f"{name}__L__{k}"] = v.numpy()
        for k, v in state.items():
            out[f"{name}__state__{k}"] = v.numpy()
        biases = []
        for lname, mod in model.named_modules():
            if isinstance(mod, (ac.QCustomBNConv2dTorch, ac.QCustomLinearTorch)):
                out[f"{name}__bA__{lname}"] = mod.get_acts_fp_bias().reshape(-1).numpy()
                out[f"{name}__bB__{lname}"] = mod.get_weights_fp_bias().reshape(-1).numpy()
                out[f"{name}__bR__{lname}"] = mod.get_res_fp_bias().reshape(-1).numpy()
                biases.append(lname)
        out[f"{name}__x_cal"], out[f"{name}__x_ev"] = x_cal.numpy(), x_ev.numpy()
        out[f"{name}__logits"] = logits.numpy()
        meta.append(dict(name=name, E=E, M=M, with_comp=wc, width_mult=0.25, input_size=32, n_class=10,
                         run_method=run_method, zero_table_ext=(E, M) == (5, 2),
                         state_keys=list(state.keys()), approx_layers=biases))
    ac.get_error_table_NN = v9.get_error_table_NN
    np.savez_compressed(os.path.join(HERE, "g8_mbv2.npz"), **out)
    return meta


# ----------------------------------------------------------------------------- G5
def qparams_for(E, M, approx_cfg, run_method):
    return dict(
        method=FPQuantizer, act_method=FPQuantizer, n_bits=8, n_bits_act=8,
        per_channel_weights=True,
        weight_range_method=RangeEstimators.current_minmax.cls, weight_range_options={},
        act_range_method=RangeEstimators.allminmax.cls, act_range_options={},
        quantize_input=True,
        fp8_kwargs=dict(maxval=None, mantissa_bits=M, set_maxval=True, learn_maxval=False,
                        learn_mantissa_bits=False, mse_include_mantissa_bits=False,
                        allow_unsigned=False),
        custom_approx_params=approx_cfg, run_method=run_method)


def gen_g5():
    out, meta = {}, []
    torch.manual_seed(2024)
    run_method = dict(approx_flag=True, quantize_after_mult_and_add=False,
                      res_quantizer_flag=True, original_quantize_res=False)
    qamaa_rm = dict(approx_flag=False, quantize_after_mult_and_add=True, res_quantizer_flag=True,
                    original_quantize_res=False)
    cases = [
        ("conv_e4m3_nocomp", (4, 3), dict(cin=8, cout=16, k=3, stride=1, pad=1, groups=1), False, True, True),
        ("qamaa_conv_e3m4", (3, 4), dict(cin=6, cout=10, k=3, stride=1, pad=1, groups=1), False, True, True),
        ("qamaa_linear_e4m3", (4, 3), dict(fin=20, fout=9), False, True, True),
        ("conv_e4m3_comp_s2", (4, 3), dict(cin=8, cout=16, k=3, stride=2, pad=1, groups=1), True, True, True),
        ("conv_e3m4_comp3", (3, 4), dict(cin=6, cout=12, k=3, stride=1, pad=0, groups=1), True, False, True),
        ("dwconv_e3m4_nocomp", (3, 4), dict(cin=8, cout=8, k=3, stride=1, pad=1, groups=8), False, True, True),
        ("conv1x1_e2m5_comp3", (2, 5), dict(cin=16, cout=8, k=1, stride=1, pad=0, groups=1), True, True, False),
        ("linear_e4m3_nocomp", (4, 3), dict(fin=32, fout=10), False, True, True),
        ("linear_e3m4_comp3", (3, 4), dict(fin=24, fout=7), True, True, True),
    ]
    for (name, (E, M), shp, wc, s2n, qbma) in cases:
        cfg = approx_params(E, M, 3, wc, True, s2n, qbma)
        rm = qamaa_rm if name.startswith("qamaa") else run_method
        qp = qparams_for(E, M, cfg, dict(rm))
        if "fin" in shp:
            mod = ac.QCustomLinearTorch(in_features=shp["fin"], out_features=shp["fout"], bias=True, **qp)
            x_cal = torch.randn(6, shp["fin"])
            x_ev = torch.randn(5, shp["fin"])
        else:
            mod = ac.QCustomBNConv2dTorch(in_channels=shp["cin"], out_channels=shp["cout"],
                                          kernel_size=shp["k"], stride=shp["stride"], padding=shp["pad"],
                                          groups=shp["groups"], bias=False, activation=nn.ReLU(), **qp)
            with torch.no_grad():
                mod.gamma.uniform_(0.5, 1.5)
                mod.beta.uniform_(-0.2, 0.2)
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 2.0)
            x_cal = torch.relu(torch.randn(2, shp["cin"], 7, 7))
            x_ev = torch.relu(torch.randn(2, shp["cin"], 7, 7))
        with torch.no_grad():
            mod.weight.normal_(0, 0.3)
            if getattr(mod, "bias", None) is not None:
                mod.bias.uniform_(-0.1, 0.1)
        state = {k: v.clone() for k, v in mod.state_dict().items()}
        mod.eval()
        mod.quantized()
        mod.estimate_ranges()
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            y_cal = mod(x_cal)
        mod.fix_ranges()
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            y_ev = mod(x_ev)
        for k, v in state.items():
            out[f"{name}__state__{k}"] = v.numpy()
        out[f"{name}__x_cal"] = x_cal.numpy()
        out[f"{name}__x_ev"] = x_ev.numpy()
        out[f"{name}__y_cal"] = y_cal.numpy()
        out[f"{name}__y_ev"] = y_ev.numpy()
        out[f"{name}__bA"] = mod.get_acts_fp_bias().reshape(-1).numpy()
        out[f"{name}__bB"] = mod.get_weights_fp_bias().reshape(-1).numpy()
        out[f"{name}__bR"] = mod.get_res_fp_bias().reshape(-1).numpy()
        meta.append(dict(name=name, E=E, M=M, shape=shp, with_comp=wc, s2n=s2n, qbma=qbma, run_method=rm,
                         state_keys=list(state.keys())))
    np.savez_compressed(os.path.join(HERE, "g5_operator.npz"), **out)
    return meta


GROUPS = dict(g1=lambda: gen_g1(), g2=lambda: gen_g2(), g3=lambda: gen_g3(), g4=lambda: gen_g4(),
              g5=lambda: gen_g5(), g6=lambda: gen_g6(), g7=lambda: gen_g7(), g8=lambda: gen_g8())


def main(argv):
    """All groups, or only the named ones (e.g. `gen_golden.py g7 g8`): meta.json keeps the other
    groups' entries."""
    torch.set_num_threads(os.cpu_count() or 1)
    names = argv or list(GROUPS)
    mpath = os.path.join(HERE, "meta.json")
    meta = {}
    if argv and os.path.exists(mpath):
        with open(mpath) as f:
            meta = json.load(f)
    meta.update(torch_version=torch.__version__, reference="revollllt/FP8_quantization@2024-11-08")
    for n in names:
        meta[n] = GROUPS[n]()
    with open(mpath, "w") as f:
        json.dump(meta, f, indent=1)
    sizes = {f: os.path.getsize(os.path.join(HERE, f)) for f in os.listdir(HERE) if f.endswith(".npz")}
    print(json.dumps(sizes))


if __name__ == "__main__":
    main(sys.argv[1:])
