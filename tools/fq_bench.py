#!/usr/bin/env python
"""Throughput of the fake-quant kernel (fp8a_fp8_quantize, per tensor) on a large fp32 tensor:
    python tools/fq_bench.py [--n 268435456] [--reps 5]
FP8A_LIB_PATH selects an alternative build (A/B of quantizer forms)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from fp8_quantization_amd.approx_ops import fp8_fake_quantize
    x = torch.randn(args.n, device="cuda:0")
    mx = torch.tensor([3.0], device="cuda:0")
    fp8_fake_quantize(x, mx, 8, 3)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fp8_fake_quantize(x, mx, 8, 3)
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    print(json.dumps(dict(n=args.n, ms=round(best, 4), gbs=round(8.0 * args.n / best / 1e6, 1),
                          lib=os.environ.get("FP8A_LIB_PATH", "default"))))


if __name__ == "__main__":
    main()
