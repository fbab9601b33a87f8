"""Operand-exponent statistics of the approx layers (design study for the matrix-core term split).

For every approx conv / linear of a bench workload (same protocol as bench.py), on a row sample:
  * the fraction of nonzero products whose magnitude falls below the result grid's smallest
    normal 2^(1 - bR) (the subnormal band / flush region of Q_R, where the term is not
    c_a c_b L(m_a, m_b));
  * the fraction of nonzero A elements that could meet such a product, per threshold rule:
    t(k) = (1 - bR) - min over a column tile of e_b(k, n) for tiles of 32 / 64 / 128 / 256 / all
    columns (small a: e_a < t(k)).
Run on the GPU box: FP8A_FUSE_QIN=0 FP8A_FUSE_BLOCK=0 python tools/unsafe_stats.py --arch resnet18
"""
import argparse
import json
import os
import sys

os.environ.setdefault("FP8A_FUSE_QIN", "0")
os.environ.setdefault("FP8A_FUSE_BLOCK", "0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def expo(t):
    """floor(log2|t|) as int32, -1000 for zeros."""
    m, e = torch.frexp(t)
    e = (e - 1).to(torch.int32)
    return torch.where(t == 0, torch.full_like(e, -1000), e)


def layer_stats(A, B, bR, rows=2048):
    g = torch.Generator(device="cpu").manual_seed(0)
    if A.shape[0] > rows:
        idx = torch.randperm(A.shape[0], generator=g)[:rows].to(A.device)
        A = A[idx]
    ea, eb = expo(A), expo(B)  # [m, K], [K, N]
    thr = 1 - int(bR)
    nz_a = (A != 0)
    nz_b = (B != 0)
    # products below 2^thr (chunks over K to bound memory)
    unsafe, nzp = 0, 0
    for k0 in range(0, A.shape[1], 64):
        a = A[:, k0:k0 + 64].abs().unsqueeze(2)
        b = B[k0:k0 + 64].abs().unsqueeze(0)
        p = a * b
        nzp += int((p != 0).sum())
        unsafe += int(((p != 0) & (p < 2.0 ** thr)).sum())
    out = dict(M=A.shape[0], K=A.shape[1], N=B.shape[1], bR=int(bR), nz_a=float(nz_a.float().mean()),
               nz_b=float(nz_b.float().mean()), unsafe_pair_frac=unsafe / max(nzp, 1))
    N = B.shape[1]
    for tile in (32, 64, 128, 256, N):
        if tile > N and tile != N:
            continue
        nt = (N + tile - 1) // tile
        ebp = torch.full((B.shape[0], nt * tile), 1000, dtype=torch.int32, device=B.device)
        ebp[:, :N] = torch.where(nz_b, eb, torch.full_like(eb, 1000))
        mins = ebp.view(B.shape[0], nt, tile).amin(dim=2)  # [K, nt]
        t = thr - mins  # small a at (m, k) for tile j: e_a < t[k, j]
        small = (ea.unsqueeze(2) < t.unsqueeze(0)) & nz_a.unsqueeze(2)
        out[f"small_a_frac_tile{tile if tile != N else 'all'}"] = float(small.float().sum() / nz_a.sum().clamp(min=1)
                                                                        / nt)
    # split both operands at one exponent: small a (e_a < tau), small b (e_b < thr - tau);
    # products not covered by (small a) u (small b) are safe.  Best tau.
    ea_nz, eb_nz = ea[nz_a], eb[nz_b]
    best = (2.0, None, 0, 0)
    for tau in range(-60, 40):
        fa = float((ea_nz < tau).float().mean())
        fb = float((eb_nz < thr - tau).float().mean())
        tot = fa + fb - fa * fb
        if tot < best[0]:
            best = (tot, tau, fa, fb)
    out.update(split_best=best[0], split_tau=best[1], split_fa=best[2], split_fb=best[3])
    # compaction cost of that split (the round-3 small-set path): per 16-row block, every row's
    # small A entries padded to the block's longest list (lanes of a wave = the block's rows), and
    # per 16-column block the same for small weights; eff = entries / padded slots
    if best[1] is not None:
        tau = best[1]
        small_a = (nz_a & (ea < tau)).sum(dim=1).float()  # [rows]
        nb = small_a.numel() // 16
        if nb:
            blk = small_a[:nb * 16].view(nb, 16)
            out["rowpad_eff_a"] = float(blk.sum() / (16 * blk.amax(dim=1)).sum().clamp(min=1))
        small_b = (nz_b & (eb < thr - tau)).sum(dim=0).float()  # [cols]
        nbb = small_b.numel() // 16
        if nbb:
            blk = small_b[:nbb * 16].view(nbb, 16)
            out["colpad_eff_b"] = float(blk.sum() / (16 * blk.amax(dim=1)).sum().clamp(min=1))
    # per-(k, 32-column block) percentile thresholds: small b = below the block's q-quantile,
    # small a = e_a < thr - (q-quantile exponent)
    for q in (0.05, 0.1, 0.2):
        nt = (N + 31) // 32
        ebf = torch.where(nz_b, eb, torch.full_like(eb, 1000)).float()
        ebp = torch.full((B.shape[0], nt * 32), 1000.0, device=B.device)
        ebp[:, :N] = ebf
        blk = ebp.view(B.shape[0], nt, 32)
        qv = torch.quantile(blk, q, dim=2, interpolation="lower")  # [K, nt]
        fb = float(((blk < qv.unsqueeze(2)) & (blk < 999)).float().sum() / nz_b.sum().clamp(min=1))
        t = thr - qv
        small = (ea.unsqueeze(2).float() < t.unsqueeze(0)) & nz_a.unsqueeze(2)
        fa = float(small.float().sum() / nz_a.sum().clamp(min=1) / nt)
        out[f"q{q}_fa"], out[f"q{q}_fb"] = fa, fb
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--expo-width", type=int, default=4)
    ap.add_argument("--mant-width", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/unsafe_stats.json")
    args = ap.parse_args()
    import bench
    from fp8_quantization_amd import approx_calculation as ac
    dev = torch.device("cuda", 0)
    cfg = dict(expo_width=args.expo_width, mant_width=args.mant_width, dnsmp_factor=3, withComp=False,
               with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    model, in_shape, _ = bench.build_workload(args.arch, cfg, 4, dev)
    model = model.to(dev).eval()
    rec = []
    orig_conv, orig_mm = ac.approx_conv2d, ac.approx_matmul

    def conv_hook(x, w, E, M, bA, bW, bR, table=None, **kw):
        if capture[0]:
            cols = F.unfold(x, w.shape[2:], dilation=kw.get("dilation", 1), padding=kw.get("padding", 0),
                            stride=kw.get("stride", 1))
            g = kw.get("groups", 1)
            if g == 1:
                A = cols.transpose(1, 2).reshape(-1, cols.shape[1])
                B = w.reshape(w.shape[0], -1).t() * 1.0
                bwv = bW.reshape(-1)
                rec.append(dict(kind="conv", shape=list(w.shape), **layer_stats(A, B, bR.reshape(-1)[0])))
        return orig_conv(x, w, E, M, bA, bW, bR, table, **kw)

    def mm_hook(x, y, E, M, bA, bB, bR, table=None, **kw):
        if capture[0] and y.shape[1] > 1:
            rec.append(dict(kind="linear", **layer_stats(x, y, bR.reshape(-1)[0])))
        return orig_mm(x, y, E, M, bA, bB, bR, table, **kw)

    capture = [False]
    ac.approx_conv2d, ac.approx_matmul = conv_hook, mm_hook
    with torch.no_grad():
        model.quantized()
        model.estimate_ranges()
        model(bench.synthetic_images(64, 1234, dev, in_shape))
        model.fix_ranges()
        capture[0] = True
        model(bench.synthetic_images(args.batch, 10, dev, in_shape))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    for r in rec:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
