"""Full-size spot checks: the BASELINE configs' largest products run at their real shapes on
the GPU (split-K, tails and all), and a random sample of outputs is checked against the CPU
oracle (which could not afford the whole product).  Same bars as test_gpu_parity.py."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests import golden_io as gio

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _grid(rng, E, M, shape, bias, zero_frac=0.0, top=8):
    emax = 2 ** E - 1
    expo = rng.integers(max(0, emax - top), emax + 1, size=shape)
    mant = rng.integers(0, 2 ** M, size=shape)
    v = np.where(expo == 0, np.ldexp(mant / 2 ** M, 1 - bias), np.ldexp(1.0 + mant / 2 ** M, expo - bias))
    v = v * rng.choice([-1.0, 1.0], size=shape)
    if zero_frac:
        v[rng.random(shape) < zero_frac] = 0.0
    return v.astype(np.float32)


def _table(E, M, name):
    return gio.load("g2_matmul.npz")[f"E{E}M{M}_table_{name}"]


@pytest.mark.parametrize("E,M,tname", [(4, 3, "nocomp"), (3, 4, "comp3")])
def test_vit_fc1_768x3072_batch512(E, M, tname):
    """BASELINE config 4: QCustomLinearTorch 768 -> 3072 on 512 x 197 tokens (M = 100864)."""
    from fp8_quantization_amd.approx_ops import approx_matmul, make_flags
    rng = np.random.default_rng(4)
    Mr, K, N = 512 * 197, 768, 3072
    bA, bR = 2 ** (E - 1) + 4, 2 ** (E - 1) + 5
    A = _grid(rng, E, M, (Mr, K), bA, zero_frac=0.3)
    W = _grid(rng, E, M, (N, K), 2 ** (E - 1) + 7)
    bB = rng.integers(2 ** (E - 1) + 6, 2 ** (E - 1) + 9, size=N).astype(np.int32)
    tab = _table(E, M, tname)
    Wd = torch.from_numpy(W).to(DEV)
    C = approx_matmul(torch.from_numpy(A).to(DEV), Wd.t(), E, M, bA, torch.from_numpy(bB).to(DEV), bR,
                      torch.as_tensor(tab), flags=make_flags(True, True, True))
    rows = np.sort(rng.choice(Mr, 48, replace=False))
    cols = np.sort(rng.choice(N, 32, replace=False))
    Cs = C[torch.from_numpy(rows).to(DEV)][:, torch.from_numpy(cols).to(DEV)].cpu().numpy()
    Cref, S = orc.matmul(A[rows], W[cols].T, E, M, bA, bB[cols], bR, tab, orc.flags_of(True, True, True),
                         with_abs=True)
    assert np.all(np.abs(Cs.astype(np.float64) - Cref) <= gio.sum_tolerance(S))


def _unfold_rows(x, kh, kw, stride, pad, picks):
    """im2col rows (c, ky, kx order) of the chosen (image, ho, wo) output pixels."""
    Bn, C, H, W = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    out = np.empty((len(picks), C * kh * kw), np.float32)
    for r, (b, ho, wo) in enumerate(picks):
        patch = xp[b, :, ho * stride:ho * stride + kh, wo * stride:wo * stride + kw]
        out[r] = patch.reshape(-1)
    return out


@pytest.mark.parametrize("cfg", [
    dict(name="resnet18 layer4.c2 b256", cin=512, cout=512, hw=7, k=3, s=1, p=1, Bn=256, E=4, M=3, t="nocomp"),
    dict(name="resnet18 conv1 b64", cin=3, cout=64, hw=224, k=7, s=2, p=3, Bn=64, E=4, M=3, t="nocomp"),
    dict(name="resnet50 layer3 3x3 E2M5 b64", cin=256, cout=256, hw=14, k=3, s=1, p=1, Bn=64, E=2, M=5, t="comp3"),
    dict(name="resnet50 layer2 1x1 E3M4 b64", cin=512, cout=128, hw=28, k=1, s=1, p=0, Bn=64, E=3, M=4, t="comp3"),
    dict(name="resnet50 layer3 3x3 E5M2 b64", cin=256, cout=256, hw=14, k=3, s=1, p=1, Bn=64, E=5, M=2, t="zero"),
    dict(name="resnet50 layer1 1x1 E5M2 b32", cin=64, cout=256, hw=56, k=1, s=1, p=0, Bn=32, E=5, M=2, t="zero"),
])
def test_conv_full_size_sampled(cfg):
    from fp8_quantization_amd.approx_ops import approx_conv2d, make_flags
    rng = np.random.default_rng(cfg["cin"] + cfg["cout"] + cfg["hw"])
    E, M, k, s, p = cfg["E"], cfg["M"], cfg["k"], cfg["s"], cfg["p"]
    bA, bR = 2 ** (E - 1) + 4, 2 ** (E - 1) + 5
    x = _grid(rng, E, M, (cfg["Bn"], cfg["cin"], cfg["hw"], cfg["hw"]), bA, zero_frac=0.5)
    w = _grid(rng, E, M, (cfg["cout"], cfg["cin"], k, k), 2 ** (E - 1) + 8)
    bW = rng.integers(2 ** (E - 1) + 7, 2 ** (E - 1) + 10, size=cfg["cout"]).astype(np.int32)
    tab = _table(E, M, cfg["t"])
    y = approx_conv2d(torch.from_numpy(x).to(DEV), torch.from_numpy(w).to(DEV), E, M, bA,
                      torch.from_numpy(bW).to(DEV), bR, torch.as_tensor(tab), flags=make_flags(True, True, True),
                      stride=(s, s), padding=(p, p))
    Ho = y.shape[2]
    picks = [(int(rng.integers(cfg["Bn"])), int(rng.integers(Ho)), int(rng.integers(Ho))) for _ in range(40)]
    chans = np.sort(rng.choice(cfg["cout"], 16, replace=False))
    rows = _unfold_rows(x, k, k, s, p, picks)
    Cref, S = orc.matmul(rows, w[chans].reshape(len(chans), -1).T, E, M, bA, bW[chans], bR, tab,
                         orc.flags_of(True, True, True), with_abs=True)
    yc = y.cpu().numpy()
    got = np.stack([yc[b, chans, ho, wo] for (b, ho, wo) in picks])
    assert np.all(np.abs(got.astype(np.float64) - Cref) <= gio.sum_tolerance(S)), cfg["name"]


def test_bench_workload_batch1024_sampled_through_fused_chain():
    """The headline's own launches: bench.py's ResNet-18 E4M3 workload (same construction,
    calibration batch and seeds) at its timed batch of 1024 images of 224 x 224, run through the
    fused / chained model path bench.py times (input quantizer inside the product, BN + ReLU in the
    store, the word-image hand-off from layer1.0.conv1 into layer1.0.conv2, the block tail in
    conv2's store).  The stem conv (M = 12.8 M rows, output 3.29 GB: the largest word image and
    split-K layout of the forward), layer1.0.conv1 and layer1.0.conv2 are checked on 40 output
    pixels x 16 channels against the oracle on the same operands: the epilogue is monotone, so the
    kernel's output must lie between the epilogue applied to ref -/+ the sum bar
    (|acc - ref| <= 1e-5 sum|v|), widened by a few fp32 roundings of the epilogue's own arithmetic."""
    import bench
    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd.approx_ops import fp8_fake_quantize
    from fp8_quantization_amd.distributed import calibrate_on_rank0

    cfg = dict(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False, with_approx=True, with_s2nn2s_opt=True,
               quant_btw_mult_accu=True)
    torch.manual_seed(0)  # (bench.run's order: seed, build with 4 BN-statistics batches, calibrate on 64 images)
    model, in_shape, _ = bench.build_workload("resnet18", cfg, 4, torch.device(DEV))
    model = model.to(DEV).eval()
    calibrate_on_rank0(model, [bench.synthetic_images(64, 1234, DEV, in_shape)], quantized=True)
    x = bench.synthetic_images(1024, 10, DEV, in_shape)
    rng = np.random.default_rng(1024)
    conv0, calls = ac.approx_conv2d, []

    def record(xin, w, E, M, bA, bW, bR, table=None, **kw):
        out = conv0(xin, w, E, M, bA, bW, bR, table, **kw)
        if len(calls) >= 3:
            return out
        y, ib = (out[0], out[1]) if isinstance(out, tuple) else (out, None)
        if kw.get("qin") is not None:  # the fused input quantizer: x arrives unquantized
            mx, nb, mb, sb = kw["qin"]
            xq, qb = fp8_fake_quantize(xin, mx, nb, mb, sb)
            assert torch.equal(qb.reshape(-1), ib.reshape(-1)), "input quantizer bias"
            bA = ib
        else:
            xq = xin
        k, s, p = w.shape[2], kw["stride"][0], kw["padding"][0]
        Bn, Cout, Ho, Wo = y.shape
        picks = [(int(rng.integers(Bn)), int(rng.integers(Ho)), int(rng.integers(Wo))) for _ in range(40)]
        chans = np.sort(rng.choice(Cout, 16, replace=False))
        rows = np.stack([torch.nn.functional.pad(xq[b], (p, p, p, p))[:, ho * s:ho * s + k, wo * s:wo * s + k]
                         .reshape(-1).cpu().numpy() for (b, ho, wo) in picks])
        ci = torch.from_numpy(chans).to(DEV)
        got = np.stack([y[b, ci, ho, wo].cpu().numpy() for (b, ho, wo) in picks])
        post = kw.get("post")
        res = None
        if post is not None and post[0] is not None:
            res = np.stack([post[0][b, ci, ho, wo].cpu().numpy() for (b, ho, wo) in picks]).astype(np.float64)
        calls.append(dict(rows=rows, w=w[ci].reshape(len(chans), -1).t().contiguous().cpu().numpy(),
                          bA=int(bA.reshape(-1)[0].item()), bW=bW.reshape(-1)[ci].cpu().numpy().astype(np.int32),
                          bR=int(bR.reshape(-1)[0].item()), table=np.ascontiguousarray(table.numpy(), np.int32),
                          flags=int(kw["flags"]), ep=kw.get("epilogue"), post=post, res=res, got=got, chans=chans,
                          chain=kw.get("chain") is not None, shape=tuple(y.shape)))
        return out

    ac.approx_conv2d = record
    try:
        with torch.no_grad():
            model(x)
    finally:
        ac.approx_conv2d = conv0
    assert len(calls) == 3 and calls[0]["shape"] == (1024, 64, 112, 112) and calls[2]["chain"]
    for i, c in enumerate(calls):
        ref, S = orc.matmul(c["rows"], c["w"], 4, 3, c["bA"], c["bW"], c["bR"], c["table"], c["flags"], with_abs=True)
        tol = gio.sum_tolerance(S)
        lo, hi = ref - tol, ref + tol
        slop = np.zeros_like(ref)
        if c["ep"] is not None:  # BN as one fma per channel, then the clamp activation
            ss, act, alo, ahi = c["ep"]
            ssn = ss.cpu().numpy().astype(np.float64)[c["chans"]]
            sc, sh = ssn[:, 0], ssn[:, 1]
            lo, hi = np.minimum(lo * sc, hi * sc) + sh, np.maximum(lo * sc, hi * sc) + sh
            slop += 2.0 ** -23 * (np.abs(ref * sc) + np.abs(sh))
            if act:
                lo, hi = np.clip(lo, alo, ahi), np.clip(hi, alo, ahi)
        post = c["post"]
        if post is not None:  # the block tail: + residual, clamp, output quantizer (all monotone)
            if c["res"] is not None:
                lo, hi = lo + c["res"], hi + c["res"]
                slop += 2.0 ** -23 * np.abs(c["res"])
            lo, hi = lo - 2 * slop, hi + 2 * slop
            slop = np.zeros_like(ref)
            if post[1]:
                lo, hi = np.clip(lo, post[2], post[3]), np.clip(hi, post[2], post[3])
            if post[4] is not None:
                mx, nb, mb, sb = post[4]
                q = lambda v: fp8_fake_quantize(torch.from_numpy(v.astype(np.float32)).to(DEV), mx, nb, mb, sb)[0] \
                    .cpu().numpy().astype(np.float64)  # noqa: E731
                lo, hi = q(np.nextafter(lo.astype(np.float32), -np.inf)), q(np.nextafter(hi.astype(np.float32), np.inf))
        got = c["got"].astype(np.float64)
        bad = (got < lo - 2 * slop) | (got > hi + 2 * slop)
        assert not bad.any(), f"layer {i} {c['shape']}: {np.count_nonzero(bad)} sampled outputs outside the bar"
