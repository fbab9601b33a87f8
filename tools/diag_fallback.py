"""Per-layer operand ranges of a bench workload and the fallback flag of every approx launch
(diagnostics; run on the GPU box with FP8A_DEBUG_FLAGS=1 so the library prints each launch's flag
word): for each approx conv / linear of one fixed-range forward, bA / bR, the weight biases, and
the binade range of the nonzero quantized operands, to name which window a falling-back layer
leaves."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mobilenet_v2")
    ap.add_argument("--expo-width", type=int, default=5)
    ap.add_argument("--mant-width", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    cfg = dict(expo_width=a.expo_width, mant_width=a.mant_width, dnsmp_factor=3, withComp=False, with_approx=True,
               with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    model, shape, _ = bench.build_workload(a.arch, cfg, 4, dev)
    model = model.to(dev).eval()
    model.quantized()
    model.estimate_ranges()
    with torch.no_grad():
        model(bench.synthetic_images(64, 1234, dev, shape))
    model.fix_ranges()
    QuantizationHijacker.fuse_input_quant = False
    conv0 = ac.approx_conv2d

    def b2s(t):
        t = t.reshape(-1).float()
        return f"{int(t.min())}..{int(t.max())}" if t.numel() > 1 else f"{int(t[0])}"

    def binades(x):
        nz = x[x != 0].abs()
        if nz.numel() == 0:
            return "all zero"
        e = torch.floor(torch.log2(nz))
        return f"2^{int(e.min())}..2^{int(e.max())}"

    idx = [0]

    def conv(x, w, E, M, bA, bW, bR, table=None, **kw):
        torch.cuda.synchronize()
        print(f"[{idx[0]}] conv x{tuple(x.shape)} w{tuple(w.shape)} g={kw.get('groups', 1)} bA={b2s(bA)} bW={b2s(bW)} "
              f"bR={b2s(bR)} |x| {binades(x)} |w| {binades(w)}", flush=True)
        idx[0] += 1
        y = conv0(x, w, E, M, bA, bW, bR, table, **kw)
        torch.cuda.synchronize()
        return y

    ac.approx_conv2d = conv
    with torch.no_grad():
        model(bench.synthetic_images(a.batch, 10, dev, shape))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
