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
