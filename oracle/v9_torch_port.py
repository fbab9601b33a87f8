"""Vectorised torch restatement of the approx_v9 op sequence (TEST / BASELINE INFRASTRUCTURE).

Only bench.py's cpu_baseline leg and tests/ use this module.  It restates, in vectorised torch
on the CPU, the same sequence of elementwise passes the reference runs per output column
(approx/approx_matmul_whole_v9.py:10-169: golden product, Q_R, subnormal masks, decompose,
exponent add, mantissa product with table gather, Q_R, sum over K), materialising the
[M, K, 1] intermediates like the reference does.  Its cost per product therefore tracks the
reference's CPU cost, which is what the "port" CPU baseline reports; its values are pinned to
the golden vectors in tests/test_torch_port_cpu.py.
"""
import torch


def _fmt(E, M, b):
    return dict(mn=2.0 ** (1 - b), mx=(2.0 ** (2 ** E - 1 - b)) * (2 - 2.0 ** (-M)), b=b, M=M,
                maxe=2 ** E - 1, maxm=2 ** M - 1)


def _dec(x, f, clip):
    fr, e = torch.frexp(x)
    sub = x.abs() < f["mn"]
    t = torch.where(sub, torch.ldexp(fr.abs(), e + (f["b"] - 1 + f["M"])),
                    torch.ldexp(fr.abs() * 2 - 1, torch.tensor(f["M"], dtype=torch.int32)))
    mant = torch.clamp(torch.round(t), max=f["maxm"]).to(torch.int32)
    expo = torch.where(sub, torch.zeros_like(e), e + (f["b"] - 1))
    if clip:
        of = (x < -f["mx"]) | (x > f["mx"])
        expo = torch.where(of, torch.full_like(expo, f["maxe"]), expo)
        mant = torch.where(of, torch.full_like(mant, f["maxm"]), mant)
    return expo, mant


def _q(x, f, clip):
    expo, mant = _dec(x, f, clip)
    ms = mant / (2 ** f["M"])
    v = torch.where(expo == 0, 2.0 ** (1 - f["b"]) * ms, 2.0 ** (expo - f["b"]) * (1 + ms))
    return v * torch.where(x < 0, -1.0, 1.0)


def column(A, bcol, E, M, bA, bB, bR, table, approx=True, s2n=True, qbma=True, gclip=False):
    """One output column: A [M, K] fp32, bcol [K, 1] -> [M, 1] (int-bias semantics)."""
    fA, fB, fR = _fmt(E, M, bA), _fmt(E, M, bB), _fmt(E, M, bR)
    g = A.unsqueeze(2) * bcol.unsqueeze(0)
    zero = g == 0
    if qbma:
        g = _q(g, fR, gclip)
    asub = A.abs() < fA["mn"]
    bsub = bcol.abs() < fB["mn"]
    a2 = torch.where(asub, A * 2 ** M, A) if s2n else A
    b2 = torch.where(bsub, bcol * 2 ** M, bcol) if s2n else bcol
    eA, mA = _dec(a2, fA, False)
    eB, mB = _dec(b2, fB, False)
    ex = eA.unsqueeze(2) + eB.unsqueeze(0) - (bA + bB - bR)
    sgn = torch.where(g < 0, -1.0, 1.0)
    mp = (1 + mA.unsqueeze(2) * 2.0 ** -M) * (1 + mB.unsqueeze(0) * 2.0 ** -M)
    if approx:
        mp = mp - 2.0 ** -M * table[mA.unsqueeze(2).long(), mB.unsqueeze(0).long()]
    v = 2.0 ** (ex - bR) * mp * sgn
    if s2n:
        v = torch.where(asub.unsqueeze(2), v / 2 ** M, v)
        v = torch.where(bsub.unsqueeze(0), v / 2 ** M, v)
        v = torch.where(zero, 0.0, v)
    else:
        norm = (eA.unsqueeze(2) > 0) & (eB.unsqueeze(0) > 0) & (g.abs() >= fR["mn"])
        v = torch.where(norm, v, g)
    if qbma:
        v = _q(v, fR, gclip)
    return v.sum(dim=1)


def matmul(A, B, E, M, bA, bB, bR, table, **flags):
    """Per-column loop, as approx_multiply drives it (approx_calculation.py:774-799)."""
    bB = [int(b) for b in (bB if hasattr(bB, "__len__") else [bB] * B.shape[1])]
    return torch.cat([column(A, B[:, i:i + 1], E, M, bA, bB[i], bR, table, **flags) for i in range(B.shape[1])],
                     dim=1)
