#!/usr/bin/env python
"""Per-layer time of the exact depthwise 3x3 (fp8a_grouped_conv2d -> dn_dw3_kernel / dn_dw3g_kernel /
dn_group_conv) on MobileNetV2's 17 depthwise geometries at one batch, against a device copy of
the same bytes (torch clone of the input: the achievable streaming rate on this box).

    python tools/dw_bench.py [--batch 512] [--dw3 1] [--target 4096] [--lds 40960] [--reps 5] [--qin]

Times with HIP events on the current stream; prints one JSON line per layer and a total with the
algorithmic bytes (input read once, output written once) per second.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (C, H_in, stride) of MobileNetV2's depthwise layers at 224 x 224, in network order
MBV2_DW = [(32, 112, 1), (96, 112, 2), (144, 56, 1), (144, 56, 2), (192, 28, 1), (192, 28, 1), (192, 28, 2),
           (384, 14, 1), (384, 14, 1), (384, 14, 1), (384, 14, 1), (576, 14, 1), (576, 14, 1), (576, 14, 2),
           (960, 7, 1), (960, 7, 1), (960, 7, 1)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        t.append(a.elapsed_time(b))
    return min(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--dw3", type=int, default=1)
    ap.add_argument("--target", type=int, default=4096)
    ap.add_argument("--lds", type=int, default=40960)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--qin", action="store_true", help="the fused config-1 form (input quantizer, BN, clamp)")
    args = ap.parse_args()
    from fp8_quantization_amd import _lib
    from fp8_quantization_amd.approx_ops import dense_conv2d_fused, grouped_conv2d
    _lib.load()
    _lib.set_option("dw3", args.dw3)
    _lib.set_option("dw_target", args.target)
    _lib.set_option("dw_lds", args.lds)
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    tot_ms = tot_copy = tot_bytes = 0.0
    for i, (C, H, s) in enumerate(MBV2_DW):
        x = torch.randn(args.batch, C, H, H, device=dev, generator=g)
        w = torch.randn(C, 1, 3, 3, device=dev, generator=g) * 0.3
        Ho = (H + 2 - 3) // s + 1
        if args.qin:
            ep = torch.stack((torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)), 1).contiguous()
            mx = torch.tensor([6.0], device=dev)
            fn = lambda: dense_conv2d_fused(x, w, C, (s, s), (1, 1), qin=(mx, 8, 3, 1), bn=(ep, 1, 0.0, 6.0))  # noqa: E731
        else:
            fn = lambda: grouped_conv2d(x, w, C, (s, s), (1, 1))  # noqa: E731
        ms = timed(fn, args.reps)
        y = torch.empty(args.batch * C * Ho * Ho, device=dev)
        src = x.reshape(-1)[: y.numel()]
        cp = 0.5 * (timed(lambda: y.copy_(src), args.reps) + timed(lambda: x.clone(), args.reps))  # (in + out) bytes moved once
        nbytes = 4.0 * (x.numel() + args.batch * C * Ho * Ho)
        tot_ms += ms
        tot_copy += cp
        tot_bytes += nbytes
        print(json.dumps(dict(layer=i, C=C, H=H, stride=s, ms=round(ms, 4), gbs=round(nbytes / ms / 1e6, 1),
                              copy_ms=round(cp, 4))))
    print(json.dumps(dict(total_ms=round(tot_ms, 3), gbs=round(tot_bytes / tot_ms / 1e6, 1),
                          copy_total_ms=round(tot_copy, 3), dw3=args.dw3, target=args.target, lds=args.lds,
                          qin=args.qin)))


if __name__ == "__main__":
    main()
