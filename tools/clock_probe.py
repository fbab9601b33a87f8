"""In-kernel clock of gemm_f8mx_kernel on the bench workload (diagnostic; MI355X_MICROARCH.md DVFS
give-back item 6): builds lib/libfp8approx_clk.so with -DFP8A_CLOCK_STAMP=1, runs >= 2 s of
back-to-back ResNet-18 forwards, then reads the s_memtime / s_memrealtime sums over a timed
window.  Usage (GPU): python tools/clock_probe.py [batch] (build it on the CPU first:
python tools/clock_probe.py --build)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLK = os.path.join(ROOT, "fp8_quantization_amd", "lib", "libfp8approx_clk.so")
sys.path.insert(0, ROOT)
if "--build" in sys.argv:
    from fp8_quantization_amd import build_native
    print(build_native.build(force=True, out=CLK, extra=build_native.EXTRA + ["-DFP8A_CLOCK_STAMP=1"]))
    sys.exit(0)
os.environ["FP8A_LIB_PATH"] = CLK

import torch  # noqa: E402

import bench  # noqa: E402
from fp8_quantization_amd import _lib  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
torch.manual_seed(0)
cfg = dict(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False, with_approx=True, with_s2nn2s_opt=True,
           quant_btw_mult_accu=True)
model, in_shape, _ = bench.build_workload("resnet18", cfg, 4, dev)
model = model.to(dev).eval()
with torch.no_grad():
    model.quantized()
    model.estimate_ranges()
    model(bench.synthetic_images(64, 1234, dev, in_shape))
    model.fix_ranges()
    x = bench.synthetic_images(batch, 10, dev, in_shape)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.5:  # warm: >= 2 s of back-to-back launches
        model(x)
    _lib.clock_stats(reset=True)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 3.0:
        model(x)
        n += 1
    st = _lib.clock_stats(reset=True)
print(dict(st, batch=batch, forwards=n, ms_per_forward=(time.perf_counter() - t0) / n * 1e3), flush=True)
