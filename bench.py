#!/usr/bin/env python
"""Headline benchmark: ImageNet-val images/s of ResNet-18 FP8 approx_v9 (BASELINE.json metric).

One step = one forward of ResNet-18 (20 approx convs + approx fc, BN, ReLU, pools, FP8
activation / weight / result quantizers) over a batch of synthetic ImageNet-shaped images
(3x224x224) already resident in HBM, in the reference's eval protocol
(run_method approx_flag + res_quantizer_flag, ranges fixed after one calibration batch),
E4M3, dnsmp_factor=3, with_s2nn2s_opt, quant_btw_mult_accu.  Random-init weights (no network
for checkpoints), synthetic data (no ImageNet here).

N>1 (torch.distributed.run, one rank per GPU, RCCL): the validation batch is sharded --
each rank runs its own B images (weak scaling) and the logits are all-gathered once per step,
as the validate driver does.

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel family, the fused
approx GEMM/conv launches (fp8a_conv2d / fp8a_matmul), timed with HIP events on the stream
they run on; `cpu_baseline` is the vectorised torch restatement of the reference's op sequence
(oracle/v9_torch_port.py, cost within ~5 % of the reference on identical inputs) on a bounded
sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ARCH_NAMES = {"resnet18": "ResNet-18", "resnet50": "ResNet-50", "mobilenet_v2": "MobileNetV2",
              "vit_fc": "ViT-B/16 fc1 (768x3072)", "vit_b16": "ViT-B/16"}
# images per GPU per step when --batch is not given.  CNNs: 512 (the reference validates at 128,
# image_net.py / click_options.py:44; inference throughput is batch-size free, and at 512 the
# small-spatial layers fill the 256 CUs: ResNet-18 11086 / 11640 / 11863 images/s at 256 / 512 /
# 768 on one box).  ViT-B/16 is BASELINE config 4, batch 512 over 8 GPUs = 64 per GPU; the vit_fc
# GEMM keeps its round-1/2 shape (256 x 197 token rows).
DEFAULT_BATCH = {"vit_b16": 64, "vit_fc": 256}
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X fp32 vector (= fp32 MFMA) peak, MI355X_MICROARCH.md


def metric_name(arch, E, M):
    """BASELINE.json's metric for the headline (ResNet-18 E4M3); the same wording for the other
    configs.  The top-1 clause is not part of it: top-1 is not measured here (no ImageNet or
    pretrained weights offline) -- see the line's ``top1_delta``."""
    fmt = "" if (E, M) == (4, 3) else f" E{E}M{M}"
    return f"ImageNet val images/sec, {ARCH_NAMES[arch]} FP8{fmt} approx_v9"


def dominant_kernel(E, M):
    """(kernel name, description) of the approx GEMM kernel the bench's format runs on (run_gemm
    in csrc/fp8approx.hip; the bench uses s2n + qbma and the withComp=False tables): the E4M3
    matrix-core form for E4M3, the tile-table kernel for E3M4 / E2M5 (their tables have no
    negative entries), the VALU tiled kernel otherwise."""
    if (E, M) == (4, 3):
        return "gemm_f8mx_kernel", ("implicit-GEMM approx conv / linear, E4M3 terms by the hardware fp8 "
                                    "conversion, codes summed on the matrix core")
    if M in (4, 5):
        return "gemm_tt_kernel", (f"implicit-GEMM approx conv / linear on the VALU, E{E}M{M} terms from a "
                                  "per-tile c_b-applied table, one multiply + magic-constant Q_R + add per product")
    return "gemm_fast_kernel", (f"implicit-GEMM approx conv / linear on the VALU, E{E}M{M} error-table "
                                "term, arithmetic Q_R")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None, help="images per GPU per step (default 512; vit_b16 64, vit_fc 256)")
    ap.add_argument("--cal-batch", type=int, default=64)
    ap.add_argument("--with-comp", action="store_true", help="withComp=True (E4M3: all-zero error table)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-columns", type=int, default=48, help="output columns per layer in the CPU sample")
    ap.add_argument("--arch", default="resnet18", choices=sorted(ARCH_NAMES),
                    help="resnet18 = the headline (BASELINE configs[1]); the others are BASELINE configs 3-5 "
                         "measured the same way (vit_b16: the whole ViT-B/16 of vit_quantized_approx; vit_fc: its "
                         "768x3072 QCustomLinearTorch alone on [B, 197, 768])")
    ap.add_argument("--bn-stats-batches", type=int, default=4,
                    help="synthetic batches that set the random-init float model's BN statistics (0 = keep the "
                         "default (0, 1) statistics)")
    ap.add_argument("--expo-width", type=int, default=4)
    ap.add_argument("--mant-width", type=int, default=3)
    args = ap.parse_args()
    if args.batch is None:
        args.batch = DEFAULT_BATCH.get(args.arch, 512)
    return args


def synthetic_images(n, seed, device, shape=(3, 224, 224)):
    g = torch.Generator(device="cpu").manual_seed(seed)
    # ImageNet-normalised statistics: roughly N(0, 1) per channel (ViT fc: token features)
    return torch.randn((n,) + tuple(shape), generator=g).to(device)


def build_workload(arch, cfg, bn_batches=0, device=None):
    """(model, per-image input shape, description) of a BASELINE config."""
    from fp8_quantization_amd import resnet_workload as rw
    bn = dict(bn_stats_batches=bn_batches, device=device)
    if arch == "resnet18":
        return rw.resnet18_approx(**bn, **cfg), (3, 224, 224), "resnet18"
    if arch == "resnet50":
        return rw.resnet50_approx(**bn, **cfg), (3, 224, 224), "resnet50"
    if arch == "mobilenet_v2":
        from fp8_quantization_amd.mobilenet_workload import mobilenet_v2_approx
        return mobilenet_v2_approx(**bn, **cfg), (3, 224, 224), "mobilenet_v2"
    if arch == "vit_b16":  # no BN: the random-init (HF initialisation) network is used as is
        from fp8_quantization_amd.vit_workload import vit_b16_approx
        return vit_b16_approx(**cfg), (3, 224, 224), ("vit_b16 (vit_quantized_approx module tree: 72 approx "
                                                      "QCustomLinearTorch on [B, 197, *] token rows + classifier)")
    from fp8_quantization_amd.approx_calculation import QCustomLinearTorch
    from fp8_quantization_amd.model_wrap import QuantizedModel

    class VitFc(QuantizedModel):  # vit_quantized_approx's intermediate dense: 768 -> 3072 on 197 tokens
        def __init__(self):
            super().__init__((1, 197, 768))
            self.fc1 = QCustomLinearTorch(in_features=768, out_features=3072, bias=True, **rw.approx_qparams(**cfg))
            self.fc1.flatten_leading_dims = True  # the reference asserts on 3-D inputs

        def forward(self, x):
            return self.fc1(x)
    return VitFc(), (197, 768), "vit_b16 fc1 (768x3072 QCustomLinearTorch, 197 tokens/image)"


PMC_FILES = ("pmc_r02b.json", "pmc_r02.json", "pmc_r01.json")


def pmc_traffic(kernel, arch, E, M, batch):
    """Per-launch HBM bytes of the approx GEMM kernel from a committed rocprofv3 PMC summary
    (profiles/pmc_<round>.json, tools/prof_summary.py) recorded for this same kernel, workload,
    format and batch (summaries without a batch field were taken at 256); None when no such
    summary exists."""
    for name in PMC_FILES:
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        if (j.get("kernel"), j.get("arch"), j.get("E"), j.get("M"), j.get("batch", 256)) == (kernel, arch, E, M, batch):
            return j.get("bytes_per_launch")
    return None


def cpu_baseline(shapes, table, cols):
    """Reference-cost CPU throughput on a bounded sample: for every distinct approx layer
    shape of ONE image, time `cols` output columns of the torch port, scale by the layer's
    column count; images/s = 1 / projected seconds per image."""
    from oracle import v9_torch_port as port
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    fa, fb = port._fmt(4, 3, 12), port._fmt(4, 3, 19)
    g = torch.Generator().manual_seed(7)
    per_img, measured, cache = 0.0, 0.0, {}
    for (_, Mi, K, N, groups) in shapes:
        key = (Mi, K)
        if key not in cache:
            A = port._q(torch.randn((Mi, K), generator=g).relu(), fa, True)
            B = port._q(torch.randn((K, cols), generator=g) * 0.05, fb, True)
            nc = min(cols, N)
            t0 = time.perf_counter()
            for c in range(nc):
                port.column(A, B[:, c:c + 1], 4, 3, 12, 19, 15, table, approx=True, s2n=True, qbma=True)
            dt = (time.perf_counter() - t0) / nc
            cache[key] = dt
            measured += dt * nc
        per_img += cache[key] * N * groups
    return dict(value=1.0 / per_img, unit="images/s", cores=threads, kind="port",
                sample=(f"1 image: up to {cols} output columns of each of {len(cache)} distinct approx layer shapes "
                        f"(torch port of the v9 op sequence, {measured:.1f} s measured), scaled by each layer's "
                        f"output-column count; {per_img:.1f} s/img projected"))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.manual_seed(0)

    import fp8_quantization_amd as fa
    from fp8_quantization_amd import approx_ops as am
    from fp8_quantization_amd.distributed import broadcast_quant_state, gather_logits
    from fp8_quantization_amd.error_tables import get_error_table_NN
    from fp8_quantization_amd.resnet_workload import approx_layer_shapes, approx_macs_per_image

    fa._lib.load()
    cfg = dict(expo_width=args.expo_width, mant_width=args.mant_width, dnsmp_factor=3, withComp=args.with_comp,
               with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    model, in_shape, arch_desc = build_workload(args.arch, cfg, args.bn_stats_batches, dev)
    model = model.to(dev).eval()

    # calibration (one batch, identical on every rank), then fixed ranges -- image_net.py:76-91
    with torch.no_grad():
        shapes, hooks = approx_layer_shapes(model)
        model.quantized()
        model.estimate_ranges()
        model(synthetic_images(args.cal_batch, 1234, dev, in_shape))
        model.fix_ranges()
        for h in hooks:
            h.remove()
        broadcast_quant_state(model, src=0)  # identical bA/bB/bR on every rank
    macs_img = approx_macs_per_image(shapes)

    x = synthetic_images(args.batch, 10 + rank, dev, in_shape)  # this rank's shard of the validation batch

    def step():
        return gather_logits(model(x))  # one RCCL all-gather of logits per step (N > 1)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        am._PROFILE = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        prof, am._PROFILE = am._PROFILE, None

    op_ms = sum(s.elapsed_time(e) for (s, e, _) in prof)
    op_macs = sum(m for (_, _, m) in prof)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    images = world * args.batch * args.steps

    if rank == 0:
        kernel, kdesc = dominant_kernel(args.expo_width, args.mant_width)
        launches = len(prof)
        avg_s = op_ms / 1e3 / launches
        achieved = 2.0 * (op_macs / launches) / avg_s / 1e12
        res = {
            "metric": metric_name(args.arch, args.expo_width, args.mant_width),
            "value": images / elapsed,
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "top1_delta": None,
            "top1_note": "not measured: ImageNet and pretrained weights are not available offline; every layer's "
                         "output is parity-checked against the oracle instead (tests/)",
            "dtype": "fp32",
            "data": "synthetic",
            "config": {
                "workload": f"{arch_desc} E{args.expo_width}M{args.mant_width} approx_v9 forward (dnsmp_factor=3, "
                            f"withComp={args.with_comp}, with_s2nn2s_opt, quant_btw_mult_accu, res_quantizer, fixed "
                            "ranges), ImageNet-shaped synthetic batch, random-init weights"
                            + (f" with BN statistics estimated on {args.bn_stats_batches} synthetic batches"
                               if args.bn_stats_batches and not args.arch.startswith("vit") else ""),
                "global_batch": world * args.batch,
                "per_gpu_batch": args.batch,
                "input_shape_per_image": list(in_shape),
                "approx_macs_per_image": macs_img,
                "parallelism": f"dp{world}",
            },
            "roofline": {
                "bound": "valu",
                "kernel": f"{kernel} ({kdesc}); timed per op with its operand pre-decode, split-K reduce and "
                          "gated exact kernels",
                "achieved": achieved,
                "peak": FP32_VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / FP32_VALU_PEAK_TFLOPS,
                "traffic": pmc_traffic(kernel, args.arch, args.expo_width, args.mant_width, args.batch),
                "algorithmic": f"2 FLOP per approx-MAC; {op_macs / launches:.4g} approx-MAC per launch avg over "
                               f"{launches} launches, {avg_s * 1e3:.3f} ms avg launch (HIP events)",
                "approx_macs_per_s": op_macs / (op_ms / 1e3),
                "gemm_share_of_step": op_ms / 1e3 / elapsed,
            },
        }
        if world == 1 and not args.no_cpu_baseline and (args.expo_width, args.mant_width) == (4, 3):
            res["cpu_baseline"] = cpu_baseline(shapes, get_error_table_NN(4, 3, args.with_comp, 3), args.cpu_columns)
            res["speedup_vs_cpu_baseline"] = res["value"] / res["cpu_baseline"]["value"]
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
