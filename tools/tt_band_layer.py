"""A ResNet-50 E2M5 layer's own operands (bench.py's workload: construction, calibration, seeds) run
through gemm_tt_kernel with the band / zero wave-tile forms off and on (option tt_band), timed with HIP
events; plus the census's prediction of the band tiles for the same operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402
import census  # noqa: E402
from fp8_quantization_amd import _lib  # noqa: E402
from fp8_quantization_amd import approx_calculation as ac  # noqa: E402
from fp8_quantization_amd.approx_ops import approx_conv2d, fp8_fake_quantize  # noqa: E402
from fp8_quantization_amd.distributed import calibrate_on_rank0  # noqa: E402

dev = torch.device("cuda", 0)
cfg = dict(expo_width=2, mant_width=5, dnsmp_factor=3, withComp=False, with_approx=True, with_s2nn2s_opt=True,
           quant_btw_mult_accu=True)
torch.manual_seed(0)
model, in_shape, _ = bench.build_workload("resnet50", cfg, 4, dev)
model = model.to(dev).eval()
calibrate_on_rank0(model, [bench.synthetic_images(64, 1234, dev, in_shape)], quantized=True)
x = bench.synthetic_images(64, 10, dev, in_shape)
calls = []
conv0 = ac.approx_conv2d


def rec(xin, w, E, M, bA, bW, bR, table=None, **kw):
    out = conv0(xin, w, E, M, bA, bW, bR, table, **kw)
    xq, ib = xin, bA
    if kw.get("qin") is not None:
        xq, ib = fp8_fake_quantize(xin, *kw["qin"])
    calls.append((xq, w, ib, bW, bR, table, dict(flags=kw["flags"], stride=kw["stride"], padding=kw["padding"],
                                                 dilation=kw["dilation"])))
    return out


ac.approx_conv2d = rec
with torch.no_grad():
    model(x)
ac.approx_conv2d = conv0
for li in (3, 13, 26, 45, 5, 11):
    xq, w, bA, bW, bR, table, kw = calls[li]
    bAi = bA._fp8a_i32 if hasattr(bA, "_fp8a_i32") else bA
    tc = census.tile_census(xq, w, int(bR.reshape(-1)[0].item()), 1, kw["stride"], kw["padding"], kw["dilation"], 2)
    ts = []
    for opt in (0, 1):
        _lib.set_option("tt_band", opt)
        for _ in range(2):
            y = approx_conv2d(xq, w, 2, 5, bAi, bW, bR, table, **kw)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            y = approx_conv2d(xq, w, 2, 5, bAi, bW, bR, table, **kw)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 5)
    print(f"layer {li} w {tuple(w.shape)} bR {int(bR.reshape(-1)[0])} bA {int(bAi.reshape(-1)[0])}: "
          f"band tiles {tc['band_only']:.3f}  tt_band 0: {ts[0]:.3f} ms  1: {ts[1]:.3f} ms", flush=True)
_lib.set_option("tt_band", 1)
