"""Census of the approx products by result-grid band.

For the matrix-core reformulation of the approx term: a term Q_R(V(m_a, m_b) c_a c_b) whose value lies
in the result grid's NORMAL range is L(m_a, m_b) c_a c_b with L = Q_R's relative rounding of V -- a
bf16-exact GEMM over a one-hot expansion of m_a (K' = 2^M K).  A term below the grid's smallest
normal 2^(1 - bR) is rounded at the fixed subnormal quantum q = 2^(1 - bR - M) instead (the "band"),
which the one-hot form gets wrong; below q / 2 it is 0.  With s = e_a + e_b (operand binades) and V
in [2^vmin, 4):
    safe  s + vmin >= 1 - bR        band  otherwise        zero  s + 2 <= log2(q) - 1
Per layer of a bench workload (bench.py's construction, calibration and seeds) this counts
  * products (nonzero operand pairs) by class, and
  * segments -- (A element, W-column tile) pairs, the unit a lockstep kernel can route -- that are
    all-safe, all-zero, or mixed (at least one band pair, or both kinds),
from per-input-channel binade histograms of the quantized input (im2col multiplicities are taken as
the output pixel count: border effects ignored) and the quantized weights' binades.

Usage (GPU box): python tools/census.py --arch resnet50 --expo-width 2 --mant-width 5 [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OFF = 300  # binade index offset (binades of fp32 values lie in [-149, 127])
NB = 2 * OFF


def binades(t):
    """floor(log2|t|) + OFF for nonzero t, -1 for zeros (int64)."""
    m, e = torch.frexp(t.float())
    return torch.where(m != 0, e.long() - 1 + OFF, torch.full_like(e.long(), -1))


def vmin_of(table, M):
    s = 1.0 + torch.arange(2 ** M, dtype=torch.float64) / 2 ** M
    V = s[:, None] * s[None, :] - table.double() / 2 ** M
    return int(torch.floor(torch.log2(V.min())).item())


def layer_census(xq, w, bR, M, table, groups, widths=(16, 64)):
    dev = xq.device
    vmin = vmin_of(table.cpu(), M)
    t_norm = 1 - int(bR)
    lq = 1 - int(bR) - M
    C = xq.shape[1]
    if w.dim() == 2:  # linear: x [rows, K], w [N, K]; A column k = feature k
        rows = xq.numel() // xq.shape[-1]
        ea = binades(xq.reshape(rows, -1))
        hist = torch.zeros((xq.shape[-1], NB), dtype=torch.float64, device=dev)
        ok = ea >= 0
        idx = torch.arange(xq.shape[-1], device=dev).expand_as(ea)
        hist.index_put_((idx[ok], ea[ok]), torch.ones(int(ok.sum()), dtype=torch.float64, device=dev),
                        accumulate=True)
        zeros_a = (~ok).sum(dim=0).double()
        B = w.t()  # [K, N]
        kc = torch.arange(B.shape[0], device=dev)
        mult = 1.0
        gsz = B.shape[1]
    else:  # conv: A column k = (c, ky, kx) of its group; values: the plane x[:, c]
        ea = binades(xq.transpose(0, 1).reshape(C, -1))
        ok = ea >= 0
        hist = torch.zeros((C, NB), dtype=torch.float64, device=dev)
        ch = torch.arange(C, device=dev)[:, None].expand_as(ea)
        hist.index_put_((ch[ok], ea[ok]), torch.ones(int(ok.sum()), dtype=torch.float64, device=dev), accumulate=True)
        zeros_a = (~ok).sum(dim=1).double()
        Cout, cin_g, kh, kw = w.shape
        cout_g = Cout // groups
        # B [K_g, Cout] per group; k -> input channel (group base + k // (kh kw))
        Bs, kcs = [], []
        for g in range(groups):
            Bs.append(w[g * cout_g:(g + 1) * cout_g].reshape(cout_g, -1).t())
            kcs.append(g * cin_g + torch.arange(cin_g * kh * kw, device=dev) // (kh * kw))
        B = torch.block_diag(*Bs) if groups > 1 else Bs[0]
        kc = torch.cat(kcs) if groups > 1 else kcs[0]
        mult = 1.0  # every A column element is gathered once per output pixel (stride / padding ignored)
        gsz = cout_g
    # per A column k: histogram over binades, suffix / prefix sums (pixels of the plane)
    H = hist[kc]  # [K, NB]
    Z = zeros_a[kc]
    suf = torch.flip(torch.cumsum(torch.flip(H, [1]), 1), [1])  # suf[:, i] = sum_{j >= i}
    pre = torch.cumsum(H, 1)  # pre[:, i] = sum_{j <= i}
    eb = binades(B)
    nzb = eb >= 0
    if groups > 1:  # block_diag zeros outside the groups are not products
        mask = torch.zeros_like(nzb)
        for g in range(groups):
            r0, c0 = g * (B.shape[0] // groups), g * gsz
            mask[r0:r0 + B.shape[0] // groups, c0:c0 + gsz] = True
        nzb &= mask
    ebo = eb - OFF  # true binade
    # products: per (k, n) with nonzero b
    thr_safe = (t_norm - vmin - ebo + OFF).clamp(0, NB)  # safe iff ea >= t_norm - vmin - eb
    thr_zero = (lq - 3 - ebo + OFF).clamp(-1, NB - 1)  # zero iff ea <= lq - 3 - eb
    sufp = torch.cat([suf, torch.zeros((suf.shape[0], 1), dtype=suf.dtype, device=dev)], 1)
    safe = torch.gather(sufp, 1, thr_safe)  # [K, N]
    prep = torch.cat([torch.zeros((pre.shape[0], 1), dtype=pre.dtype, device=dev), pre], 1)
    zero = torch.gather(prep, 1, thr_zero + 1)
    nzA = H.sum(1, keepdim=True).expand_as(safe)
    nzbf = nzb.double()
    prod = dict(nonzero=float((nzA * nzbf).sum() * mult), safe=float((safe * nzbf).sum() * mult),
                zero=float((zero * nzbf).sum() * mult))
    prod["band"] = prod["nonzero"] - prod["safe"] - prod["zero"]
    segs = {}
    for W in widths:
        ncol = B.shape[1]
        nt = (ncol + W - 1) // W
        pad = nt * W - ncol
        big = torch.iinfo(torch.int64).max // 4
        e_lo = torch.where(nzb, ebo, torch.full_like(ebo, big))
        e_hi = torch.where(nzb, ebo, torch.full_like(ebo, -big))
        if pad:
            e_lo = torch.cat([e_lo, torch.full((e_lo.shape[0], pad), big, device=dev, dtype=e_lo.dtype)], 1)
            e_hi = torch.cat([e_hi, torch.full((e_hi.shape[0], pad), -big, device=dev, dtype=e_hi.dtype)], 1)
        mn = e_lo.reshape(e_lo.shape[0], nt, W).min(2).values
        mx = e_hi.reshape(e_hi.shape[0], nt, W).max(2).values
        live = mn < big // 2  # the (k, tile) has a nonzero weight
        ts = (t_norm - vmin - mn + OFF).clamp(0, NB)
        tz = (lq - 3 - mx + OFF).clamp(-1, NB - 1)
        s_safe = torch.gather(sufp, 1, torch.where(live, ts, torch.zeros_like(ts)))
        s_zero = torch.gather(prep, 1, torch.where(live, tz + 1, torch.zeros_like(tz)))
        nA = H.sum(1, keepdim=True).expand_as(s_safe)
        livef = live.double()
        tot = float((nA * livef).sum())
        segs[W] = dict(nonzero_a_segments=tot, all_safe=float((s_safe * livef).sum()),
                       all_zero=float((s_zero * livef).sum()))
        segs[W]["mixed"] = tot - segs[W]["all_safe"] - segs[W]["all_zero"]
    return dict(vmin=vmin, t_norm=t_norm, log2_q=lq, products=prod, segments=segs,
                zero_a_fraction=float(Z.sum() / (Z.sum() + H.sum())))


def tile_census(xq, w, bR, groups, stride, padding, dilation, kblk, rowblk=64, colblk=16):
    """Fraction of the tile-table kernels' wave-tiles (rowblk consecutive output rows x kblk
    consecutive K-steps x colblk columns) whose products all lie below the result grid's smallest
    normal 2^(1 - bR) -- where the Q_R rounding constant is the fixed cmin (a 4-op loop instead of
    7, gemm_tt.h) -- and whose products all lie at or above it (6 ops, no max)."""
    import torch.nn.functional as F
    if w.dim() == 2:
        A = xq.reshape(-1, xq.shape[-1])
        Bs = [w.t()]
        As = [A]
    else:
        cin_g, cout_g = xq.shape[1] // groups, w.shape[0] // groups
        As, Bs = [], []
        for g in range(groups):
            cols = F.unfold(xq[:, g * cin_g:(g + 1) * cin_g], w.shape[2:], dilation=dilation, padding=padding,
                            stride=stride)
            As.append(cols.transpose(1, 2).reshape(-1, cols.shape[1]))
            Bs.append(w[g * cout_g:(g + 1) * cout_g].reshape(cout_g, -1).t())
    band = normal = total = 0.0
    t = 1 - int(bR)
    for A, B in zip(As, Bs):
        ea = binades(A) - OFF
        ea = torch.where(ea < -OFF, torch.full_like(ea, -10 ** 6), ea)  # zeros never raise the max
        eb = binades(B) - OFF
        eb = torch.where(eb < -OFF, torch.full_like(eb, -10 ** 6), eb)
        M_, K_ = ea.shape
        N_ = eb.shape[1]
        pm, pk, pn = (-M_) % rowblk, (-K_) % kblk, (-N_) % colblk
        big = 10 ** 6
        ea_lo = torch.where(ea < -big // 2, torch.full_like(ea, big), ea)  # zeros never lower the min
        eb_lo = torch.where(eb < -big // 2, torch.full_like(eb, big), eb)
        ea = F.pad(ea, (0, pk, 0, pm), value=-big)
        ea_lo = F.pad(ea_lo, (0, pk, 0, pm), value=big)
        eb = F.pad(eb, (0, pn, 0, pk), value=-big)
        eb_lo = F.pad(eb_lo, (0, pn, 0, pk), value=big)
        Mb, Kb, Nb = ea.shape[0] // rowblk, ea.shape[1] // kblk, eb.shape[1] // colblk
        amax = ea.reshape(Mb, rowblk, Kb, kblk).amax(dim=(1, 3))
        amin = ea_lo.reshape(Mb, rowblk, Kb, kblk).amin(dim=(1, 3))
        bmax = eb.reshape(Kb, kblk, Nb, colblk).amax(dim=(1, 3))
        bmin = eb_lo.reshape(Kb, kblk, Nb, colblk).amin(dim=(1, 3))
        for i0 in range(0, Mb, 4096):  # (chunks: [Mb, Kb, Nb] booleans)
            hi = amax[i0:i0 + 4096, :, None] + bmax[None] + 2
            lo = amin[i0:i0 + 4096, :, None] + bmin[None] - 1  # V >= 1/2 for the tables here (vmin >= -1)
            band += float((hi <= t).sum())
            normal += float((lo >= t).sum())
            total += float(hi.numel())
    return dict(band_only=band / max(total, 1), normal_only=normal / max(total, 1), wave_tiles=total)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--expo-width", type=int, default=2)
    ap.add_argument("--mant-width", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default=None)
    ap.add_argument("--tiles", action="store_true", help="also the tile-table kernels' wave-tile census")
    ap.add_argument("--tile-batch", type=int, default=8)
    args = ap.parse_args(argv)
    import bench
    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd.approx_ops import fp8_fake_quantize
    from fp8_quantization_amd.distributed import calibrate_on_rank0
    dev = torch.device("cuda", 0)
    E, M = args.expo_width, args.mant_width
    cfg = dict(expo_width=E, mant_width=M, dnsmp_factor=3, withComp=False, with_approx=True, with_s2nn2s_opt=True,
               quant_btw_mult_accu=True)
    torch.manual_seed(0)
    model, in_shape, _ = bench.build_workload(args.arch, cfg, 4, dev)
    model = model.to(dev).eval()
    calibrate_on_rank0(model, [bench.synthetic_images(64, 1234, dev, in_shape)], quantized=True)
    x = bench.synthetic_images(args.batch, 10, dev, in_shape)
    layers = []
    conv0, mm0 = ac.approx_conv2d, ac.approx_matmul

    def conv(xin, w, E_, M_, bA, bW, bR, table=None, **kw):
        out = conv0(xin, w, E_, M_, bA, bW, bR, table, **kw)
        xq = xin
        if kw.get("qin") is not None:
            mx, nb, mb, sb = kw["qin"]
            xq = fp8_fake_quantize(xin, mx, nb, mb, sb)[0]
        c = layer_census(xq, w, int(bR.reshape(-1)[0].item()), M_, table, kw.get("groups", 1))
        if args.tiles:
            xs = xq[:args.tile_batch]
            c["tiles"] = tile_census(xs, w, int(bR.reshape(-1)[0].item()), kw.get("groups", 1), kw["stride"],
                                     kw["padding"], kw["dilation"], 2 if M_ == 5 else 4)
        c.update(kind="conv", shape=list(w.shape), groups=kw.get("groups", 1),
                 macs=float(out[0].numel() if isinstance(out, tuple) else out.numel()) * w[0].numel())
        layers.append(c)
        return out

    def mm(a, b, E_, M_, bA, bB, bR, table=None, **kw):
        out = mm0(a, b, E_, M_, bA, bB, bR, table, **kw)
        c = layer_census(a, b.t(), int(bR.reshape(-1)[0].item()), M_, table, 1)
        if args.tiles:
            c["tiles"] = tile_census(a, b.t(), int(bR.reshape(-1)[0].item()), 1, None, None, None, 2 if M_ == 5 else 4)
        c.update(kind="mm", shape=[b.shape[1], b.shape[0]], groups=1, macs=float(a.shape[0] * b.shape[0] * b.shape[1]))
        layers.append(c)
        return out

    from fp8_quantization_amd import model_wrap
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    ac.approx_conv2d, ac.approx_matmul = conv, mm
    QuantizationHijacker.fuse_input_quant = True
    model_wrap.FUSE_BLOCK = True
    ac.ApproxLinearMixin.fuse_linear_block = False  # (the linear's operands through approx_matmul)
    with torch.no_grad():
        model(x)
    tot = {k: 0.0 for k in ("nonzero", "safe", "band", "zero")}
    seg = {W: {k: 0.0 for k in ("nonzero_a_segments", "all_safe", "all_zero", "mixed")} for W in (16, 64)}
    for c in layers:
        for k in tot:
            tot[k] += c["products"][k]
        for W in seg:
            for k in seg[W]:
                seg[W][k] += c["segments"][W][k]
    summary = dict(arch=args.arch, E=E, M=M, batch=args.batch, layers=len(layers),
                   products={k: v / tot["nonzero"] for k, v in tot.items() if k != "nonzero"},
                   segments={W: {k: v / s["nonzero_a_segments"] for k, v in s.items() if k != "nonzero_a_segments"}
                             for W, s in seg.items()},
                   zero_a_fraction=sum(c["zero_a_fraction"] for c in layers) / max(1, len(layers)))
    if args.tiles:  # MAC-weighted over the layers
        wsum = sum(c["macs"] for c in layers)
        summary["wave_tiles"] = {k: sum(c["tiles"][k] * c["macs"] for c in layers) / wsum
                                 for k in ("band_only", "normal_only")}
    print(json.dumps(summary))
    for i, c in enumerate(layers):
        p = c["products"]
        s64 = c["segments"][64]
        print(f"{i:3d} {c['kind']} {c['shape']} g{c['groups']} bRnorm={c['t_norm']} vmin={c['vmin']} "
              f"prod safe {p['safe'] / max(p['nonzero'], 1):.3f} band {p['band'] / max(p['nonzero'], 1):.3f} "
              f"zero {p['zero'] / max(p['nonzero'], 1):.3f} | seg64 safe {s64['all_safe'] / max(s64['nonzero_a_segments'], 1):.3f} "
              f"mixed {s64['mixed'] / max(s64['nonzero_a_segments'], 1):.3f}"
              + (f" | tiles band {c['tiles']['band_only']:.3f} normal {c['tiles']['normal_only']:.3f}" if "tiles" in c else ""))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(dict(summary=summary, layers=layers), f)


if __name__ == "__main__":
    main()
