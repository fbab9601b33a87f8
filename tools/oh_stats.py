"""One-hot path diagnostics on the benchmark network (GPU): candidate entries per product,
excluded weights, nonempty segments, and the per-kernel split of one forward (HIP events)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from fp8_quantization_amd import _lib  # noqa: E402
from fp8_quantization_amd.resnet_workload import approx_layer_shapes, approx_macs_per_image  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda", 0)
torch.manual_seed(0)
cfg = dict(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False, with_approx=True, with_s2nn2s_opt=True,
           quant_btw_mult_accu=True)
model, in_shape, _ = bench.build_workload(arch, cfg, 4, dev)
model = model.to(dev).eval()
shapes, hooks = approx_layer_shapes(model)
with torch.no_grad():
    model.quantized()
    model.estimate_ranges()
    model(bench.synthetic_images(64, 1234, dev, in_shape))
    model.fix_ranges()
for h in hooks:
    h.remove()
x = bench.synthetic_images(batch, 10, dev, in_shape)
with torch.no_grad():
    model(x)
    _lib.set_option("oh_stats", 1)
    _lib.debug_stats(reset=True)
    model(x)
    st = _lib.debug_stats(reset=True)
    _lib.set_option("oh_stats", 0)
    prods = approx_macs_per_image(shapes) * batch
    print(arch, "batch", batch, "products", prods, st, "entries/product %.4f" % (st["entries"] / prods),
          "nonempty seg frac %.3f" % (st["segments_nonempty"] / max(1, st["segments"])), flush=True)
    for corr in (1, 0):
        _lib.set_option("oh_correct", corr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            model(x)
        torch.cuda.synchronize()
        print("oh_correct", corr, "ms/forward %.2f" % ((time.perf_counter() - t0) / 3 * 1e3), flush=True)
    _lib.set_option("oh_correct", 1)
    _lib.set_option("one_hot", 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        model(x)
    torch.cuda.synchronize()
    print("f8mx ms/forward %.2f" % ((time.perf_counter() - t0) / 3 * 1e3), flush=True)
