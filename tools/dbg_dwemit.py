"""Which MobileNetV2 launches request / emit a word image (the chain's requests, per layer), on the GPU."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fp8_quantization_amd import chain
from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx

DEV = "cuda:0"
torch.manual_seed(5)
m = mobilenet_v2_approx(input_size=64, n_class=100, bn_stats_batches=1, device=DEV, expo_width=4, mant_width=3).to(DEV).eval()
g = torch.Generator().manual_seed(6)
m.quantized()
m.estimate_ranges()
with torch.no_grad():
    m(torch.randn((2, 3, 64, 64), generator=g).to(DEV))
m.fix_ranges()
x = torch.randn((3, 3, 64, 64), generator=g).to(DEV)
log = []
orig = chain.WordChain.request


def request(self, layer, xx, qin):
    out = orig(self, layer, xx, qin)
    nxt = self.next_layer
    nq = nxt.chain_input_quantizer() if nxt is not None else None
    wants = nxt.chain_wants_image() if nq is not None else None
    log.append((layer.groups, layer.in_channels, layer.out_channels,
                None if nxt is None else (nxt.groups, nxt.out_channels), nq is not None, wants,
                None if out is None or out[1] is None else out[1][-1], out is not None and out[0] is not None))
    return out


chain.WordChain.request = request
with torch.no_grad():
    m(x)
torch.cuda.synchronize()
for r in log:
    print(r)
