"""Diagnostics: which launches of a captured MobileNetV2 E5M2 forward see stale flag words on replay
(every launch's workspace is kept; its first word is the launch's final flag word)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_graph import _calibrated  # noqa: E402
from fp8_quantization_amd import _lib, approx_ops  # noqa: E402
from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx  # noqa: E402

DEV = "cuda:0"
_lib.load()
torch.manual_seed(1)
m = mobilenet_v2_approx(input_size=64, n_class=100, bn_stats_batches=1, device=DEV, expo_width=5, mant_width=2,
                        withComp=False).to(DEV).eval()
x = _calibrated(m, (3, 64, 64), 2)
wss = []
ws0 = approx_ops._workspace


def ws_rec(device, nbytes):
    t = ws0(device, nbytes)
    wss.append(t)
    return t


with torch.no_grad():
    gs = torch.cuda.Stream()
    gs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(gs):
        for _ in range(2):
            m(x)
    torch.cuda.current_stream().wait_stream(gs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    approx_ops._workspace = ws_rec
    with torch.cuda.graph(g, stream=gs, capture_error_mode="thread_local"):
        out = m(x)
    approx_ops._workspace = ws0
    print("launches with a workspace:", len(wss), flush=True)
    ref = m(x)
    torch.cuda.synchronize()
    for i in range(3):
        for w in wss:
            w[:64].fill_(0xAB)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        fl = [int(w[:4].view(torch.int32).item()) if w.numel() >= 4 else None for w in wss]
        print("replay", i, torch.equal(ref, out), _lib.fallback_stats(reset=True), flush=True)
        print("   nonzero flag words:", [(j, f) for j, f in enumerate(fl) if f], flush=True)
        print("   sizes:", [(j, wss[j].numel()) for j, f in enumerate(fl) if f], flush=True)
