#!/usr/bin/env python
"""Headline benchmark: ImageNet-val images/s of ResNet-18 FP8 approx_v9 (BASELINE.json metric).

One step = one forward of ResNet-18 (20 approx convs + approx fc, BN, ReLU, pools, FP8
activation / weight / result quantizers) over a batch of synthetic ImageNet-shaped images
(3x224x224) already resident in HBM, in the reference's eval protocol
(run_method approx_flag + res_quantizer_flag, ranges fixed after one calibration batch),
E4M3, dnsmp_factor=3, with_s2nn2s_opt, quant_btw_mult_accu.  Random-init weights (no network
for checkpoints), synthetic data (no ImageNet here).

N>1 (one rank per GPU, RCCL; under torch.distributed.run, or `--gpus N` alone, which spawns the N
ranks itself before anything touches the GPU): the validation batch is sharded -- each rank runs
its own B images (weak scaling) and the logits are all-gathered once per step, as the validate
driver does.

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
# images per GPU per step: ResNet-18 (the headline) at 1024 -- measured on one box 11677 / 11948 /
# 12062 images/s at 512 / 768 / 1024 (the 7x7 layers' last tile wave and the split-K reductions
# amortise); ViT-B/16 at 64 (config 4's 512 over 8 GPUs)
DEFAULT_BATCH = {"resnet18": 1024, "vit_b16": 64, "vit_fc": 256}
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X fp32 vector (= fp32 MFMA) peak, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0  # HBM3E spec, MI355X_MICROARCH.md
FP8_MFMA_PEAK_TFLOPS = 5000.0  # dense fp8 MFMA, MI355X_MICROARCH.md


def metric_name(arch, E, M, v5=False, no_approx=False):
    """BASELINE.json's metric for the headline (ResNet-18 E4M3); the same wording for the other
    configs.  The top-1 clause is not part of it: top-1 is not measured here (no ImageNet or
    pretrained weights offline) -- see the line's ``top1_delta``."""
    fmt = "" if (E, M) == (4, 3) else f" E{E}M{M}"
    if no_approx:
        return f"ImageNet val images/sec, {ARCH_NAMES[arch]} FP8{fmt} PTQ (approx off, exact product)"
    return f"ImageNet val images/sec, {ARCH_NAMES[arch]} FP8{fmt} " + ("approx_v5 OFUF" if v5 else "approx_v9")


def dominant_kernel(E, M, v5=False):
    """(kernel name, description) of the approx GEMM kernel the bench's format runs on (run_gemm
    in csrc/fp8approx.hip; the bench uses s2n + qbma and the withComp=False tables): the E4M3
    matrix-core form for E4M3 and E5M2 (bf8 conversion), the packed-f16 tile-table kernel for
    E3M4 (gemm_tt16_kernel on every K >= 256 layer; gemm_tt_kernel<4> on the short-K ones), the
    f32 tile-table kernel for E2M5, the v5 matrix-core form for E5M2 v5 with the adder wrap, the VALU
    tiled kernel otherwise."""
    if v5 and (E, M) == (5, 2):
        return "gemm_v5mx_kernel", ("implicit-GEMM approx conv / linear, E5M2 v5 integer-adder terms as packed 16-bit "
                                    "code arithmetic, the codes' bf16 bits summed on the matrix core")
    if v5:
        return "gemm_fast_kernel", f"implicit-GEMM approx conv / linear on the VALU, E{E}M{M} v5 integer-adder terms"
    if (E, M) in ((4, 3), (5, 2)):
        cvt = "fp8 (e4m3)" if (E, M) == (4, 3) else "bf8 (e5m2)"
        return "gemm_f8mx_kernel", (f"implicit-GEMM approx conv / linear, E{E}M{M} terms by the hardware {cvt} "
                                    "conversion, codes summed on the matrix core")
    if (E, M) == (3, 4):
        return "gemm_tt16_kernel", ("implicit-GEMM approx conv / linear, E3M4 terms in packed f16 from a per-tile "
                                    "c_b-applied table, summed on the matrix core (gemm_tt_kernel<4> on K < 256)")
    if M in (4, 5):
        return "gemm_tt_kernel", (f"implicit-GEMM approx conv / linear on the VALU, E{E}M{M} terms from a "
                                  "per-tile c_b-applied table, one multiply + magic-constant Q_R + add per product")
    return "gemm_fast_kernel", (f"implicit-GEMM approx conv / linear on the VALU, E{E}M{M} error-table "
                                "term, arithmetic Q_R")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a launcher's WORLD_SIZE, N > 1 spawns the N ranks itself")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu = the gloo rehearsal of the multi-rank flow (tests; approx ops need stand-ins)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1 on GPUs: nccl (= RCCL over xGMI, the product) or gloo (host-staged collectives: "
                         "the one-GPU rehearsal of the N-rank flow, with --share-device)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal of N ranks on one leased GPU; needs --dist-backend gloo)")
    ap.add_argument("--dump-logits", default=None,
                    help="after the timed steps, one more (untimed) step; rank 0 saves its gathered logits "
                         "there (.npy; tests)")
    ap.add_argument("--shard-seed", type=int, default=None,
                    help="seed offset of this process's input shard (default: its rank); lets a world-1 run "
                         "reproduce rank r's shard")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None, help="images per GPU per step (default 512; resnet18 1024, vit_b16 64, vit_fc 256)")
    ap.add_argument("--cal-batch", type=int, default=64)
    ap.add_argument("--with-comp", action="store_true", help="withComp=True (E4M3: all-zero error table)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="time eager forwards (default on a GPU: the forward captured once into a HIP graph, each "
                         "timed step one replay of it -- every kernel still runs; the launch gaps go)")
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
    ap.add_argument("--no-approx", action="store_true",
                    help="approx_flag off (BASELINE config 1: the reference's canonical --no-approx_flag "
                         "--original-quantize-res PTQ run): the exact products on the fp8 matrix core")
    ap.add_argument("--v5-ofuf", action="store_true",
                    help="the opt-in v5 integer-adder mode with sim_hw_add_OFUF, with_OF_opt and with_UF_opt live "
                         "(BASELINE config 3's switches, which v9 ignores: SURVEY F2)")
    args = ap.parse_args(argv)
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


def pmc_files():
    """Committed PMC summaries, newest round first (profiles/pmc_r<NN>[...].json)."""
    import glob
    return sorted((os.path.basename(f) for f in glob.glob(os.path.join(ROOT, "profiles", "pmc_r*.json"))),
                  key=lambda n: (n[5:7], n), reverse=True)


def pmc_summary(kernel, arch, E, M, batch, strict=False):
    """(file name, summary dict) of the newest committed PMC summary recorded for this kernel,
    workload, format and batch (profiles/pmc_r<round>*.json, tools/prof_summary.py); the workload's
    other-kernel summary when not strict; (None, {}) when there is none."""
    found = {}
    for name in pmc_files():
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        if (j.get("arch"), j.get("E"), j.get("M"), j.get("batch", 256)) == (arch, E, M, batch):
            found.setdefault(j.get("kernel"), (name, j))
    if kernel in found or strict:
        return found.get(kernel, (None, {}))
    return next(iter(found.values()), (None, {}))


def pmc_traffic(kernel, arch, E, M, batch, strict=False):
    """Per-launch HBM bytes of the approx GEMM kernel from a committed rocprofv3 PMC summary
    (profiles/pmc_r<round>*.json, tools/prof_summary.py) recorded for this same kernel, workload,
    format and batch (summaries without a batch field were taken at 256); None when no such
    summary exists."""
    found = {}
    for name in pmc_files():
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        if (j.get("arch"), j.get("E"), j.get("M"), j.get("batch", 256)) == (arch, E, M, batch):
            found.setdefault(j.get("kernel"), j.get("bytes_per_launch"))
    # the named kernel's summary, else the one recorded for this workload (E3M4 on MobileNetV2:
    # its short-K layers run gemm_tt_kernel<4>, which dominates there)
    if kernel in found or strict:
        return found.get(kernel)
    return next(iter(found.values()), None)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(shapes, table, cols):
    """Reference-cost CPU throughput on a bounded sample: for every distinct approx layer
    shape of ONE image, time `cols` output columns of the torch port, scale by the layer's
    column count; images/s = 1 / projected seconds per image.  The projection is checked on
    the cheapest distinct layer, timed end to end (all its columns).  Threads: every core the
    process may use, capped by OMP_NUM_THREADS when set (the GPU box's CPU share)."""
    from oracle import v9_torch_port as port
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(avail, omp) if omp > 0 else avail)
    torch.set_num_threads(threads)
    fa, fb = port._fmt(4, 3, 12), port._fmt(4, 3, 19)
    g = torch.Generator().manual_seed(7)
    per_img, measured, cache, ops = 0.0, 0.0, {}, {}
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
            ops[key] = (A, N * groups)
            measured += dt * nc
        per_img += cache[key] * N * groups
    # the projection on one whole layer: the cheapest distinct shape, every output column
    convs = {k: v for k, v in ops.items() if k[0] > 1} or ops  # (a conv layer when there is one)
    (Mi, K), (A, ncol) = min(convs.items(), key=lambda kv: kv[1][0].numel() * kv[1][1])
    B = port._q(torch.randn((K, ncol), generator=g) * 0.05, fb, True)
    t0 = time.perf_counter()
    for c in range(ncol):
        port.column(A, B[:, c:c + 1], 4, 3, 12, 19, 15, table, approx=True, s2n=True, qbma=True)
    full = time.perf_counter() - t0
    return dict(value=1.0 / per_img, unit="images/s", cores=threads, kind="port",
                cpu_model=cpu_model(), cpu_count=os.cpu_count(),
                sample=(f"1 image: up to {cols} output columns of each of {len(cache)} distinct approx layer shapes "
                        f"(torch port of the v9 op sequence, {measured:.1f} s measured), scaled by each layer's "
                        f"output-column count; {per_img:.1f} s/img projected"),
                full_layer_check=dict(shape=[Mi, K, ncol], measured_s=full, projected_s=cache[(Mi, K)] * ncol,
                                      ratio=full / (cache[(Mi, K)] * ncol)))


CHECK_REPLAYS = 3  # replays compared bit for bit with the eager forward before timing


def capture_forward(model, x, warm, sync, fallback_stats=None):
    """The forward captured into one HIP graph (torch.cuda.CUDAGraph over hipGraph) on a side
    stream warmed by `warm` eager forwards first (torch's allocator settles there; captured
    launches keep their fallback flags in their own workspace, include/fp8approx.h, so the graph
    never depends on the library's per-stream flag arena); returns (info, replay) where replay()
    runs the captured forward and all-gathers its logits.  Each of CHECK_REPLAYS replays must
    equal an eager forward bit for bit and leave the same fallback counters as that eager forward
    (a replay that met stale flag words would recompute units it need not), else (or if capture
    fails) info["captured"] is False and the caller times eager forwards."""
    from fp8_quantization_amd.distributed import gather_logits
    info = {"captured": False}
    try:
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(gs):
            for _ in range(max(1, warm)):
                model(x)
        torch.cuda.current_stream().wait_stream(gs)
        sync()
        graph = torch.cuda.CUDAGraph()
        # thread_local: other threads' HIP calls (the process group's watchdog on N > 1 ranks) stay
        # legal while this thread captures
        with torch.cuda.graph(graph, stream=gs, capture_error_mode="thread_local"):
            out = model(x)
        fb = fallback_stats or (lambda reset=False: {})
        fb(reset=True)
        ref = model(x)
        sync()
        fb_eager = fb(reset=True)
        same, fb_same = True, True
        for _ in range(CHECK_REPLAYS):
            graph.replay()
            sync()
            same &= bool(torch.equal(ref.view(torch.int32), out.view(torch.int32)))
            fb_same &= fb(reset=True) == fb_eager
        info.update(captured=same and fb_same, replay_matches_eager_bitwise=same, checked_replays=CHECK_REPLAYS,
                    replay_fallback_matches_eager=fb_same, eager_fallback=fb_eager)
        if not (same and fb_same):
            return info, None
    except Exception as e:  # noqa: BLE001 -- report and time eager forwards instead
        import traceback
        info["error"] = f"{type(e).__name__}: {e}"[:300]
        info["where"] = "".join(traceback.format_tb(e.__traceback__)[-4:])[-1500:]
        sync()
        return info, None

    def replay():
        graph.replay()
        return gather_logits(out)
    info["note"] = ("timed steps = replays of the captured forward (every kernel of the forward runs each step); "
                    "roofline / fallback / path figures from the same number of eager steps after them")
    return info, replay


def run(args, dev, rank=0, world=1):
    """The benchmark on an initialised process group (world > 1) or alone; returns rank 0's
    JSON dict (None on the other ranks).  On a CPU device (the gloo rehearsal in
    tests/test_distributed_cpu.py, approx ops replaced by stand-ins) the control flow is the same
    and the HIP-event roofline is omitted."""
    cuda = dev.type == "cuda"
    from fp8_quantization_amd.distributed import comm_device
    comm_dev = comm_device() if world > 1 else dev

    def sync():
        if cuda:
            torch.cuda.synchronize()
    torch.manual_seed(0)

    import fp8_quantization_amd as fa
    from fp8_quantization_amd import approx_ops as am
    from fp8_quantization_amd.distributed import calibrate_on_rank0, gather_logits
    from fp8_quantization_amd.error_tables import get_error_table_NN
    from fp8_quantization_amd.resnet_workload import approx_layer_shapes, approx_macs_per_image

    fa._lib.load()
    # formats the reference has no error table for (E5M2, configs 3 / 5) run with the opt-in
    # all-zero table (approx_qparams: zero_table_ext)
    cfg = dict(expo_width=args.expo_width, mant_width=args.mant_width, dnsmp_factor=3, withComp=args.with_comp,
               with_approx=True, with_s2nn2s_opt=True, quant_btw_mult_accu=True)
    if args.v5_ofuf:
        cfg.update(approx_version=5, withComp=True, sim_hw_add_OFUF=True, with_OF_opt=True, with_UF_opt=True)
    if args.no_approx:  # scripts/image_net.sh:42-45 (--no-approx_flag --original-quantize-res)
        cfg.update(run_method=dict(approx_flag=False, quantize_after_mult_and_add=False, res_quantizer_flag=True,
                                   original_quantize_res=True))
    model, in_shape, arch_desc = build_workload(args.arch, cfg, args.bn_stats_batches, dev)
    model = model.to(dev).eval()

    # calibration (one batch) on rank 0 alone, then fixed ranges -- image_net.py:76-91; the other
    # ranks take rank 0's model state and FP8 ranges by broadcast (identical bA/bB/bR everywhere)
    shapes, hooks = approx_layer_shapes(model)
    calibrate_on_rank0(model, [synthetic_images(args.cal_batch, 1234, dev, in_shape)] if rank == 0 else [],
                       quantized=True)
    for h in hooks:
        h.remove()
    macs_img = approx_macs_per_image(shapes)  # (rank 0's calibration pass recorded the shapes)

    shard = rank if args.shard_seed is None else args.shard_seed
    x = synthetic_images(args.batch, 10 + shard, dev, in_shape)  # this rank's shard of the validation batch

    def step():
        return gather_logits(model(x))  # one RCCL all-gather of logits per step (N > 1)

    def instrumented(fn):
        """K steps of fn with the per-op HIP events (approx_ops._PROFILE), the product kernels'
        HIP events (fp8a_kernel_timing) and the fallback / path counters on; returns the wall
        time between the two barrier + synchronize brackets and the op events."""
        sync()
        if world > 1:
            dist.barrier()
        am._PROFILE = [] if cuda else None
        if cuda:
            fa._lib.fallback_stats(reset=True)  # (synchronises: outside the timed region)
            fa._lib.path_stats(reset=True)
            fa._lib.dense_stats(reset=True)
            fa._lib.kernel_time(reset=True)
            fa._lib.kernel_timing(True)  # HIP events around each GEMM's product kernel (fp8a_kernel_timing)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        sync()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        pr, am._PROFILE = am._PROFILE or [], None
        if cuda:
            fa._lib.kernel_timing(False)
        return el, pr

    graph_info = None
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        if cuda and not args.no_graph:
            graph_info, replay = capture_forward(model, x, args.warmup, sync, fa._lib.fallback_stats)
            if world > 1:  # every rank replays or none does: the timed loops must issue the same collectives
                ok = torch.tensor([1 if graph_info.get("captured") else 0], dtype=torch.int32, device=comm_dev)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                graph_info["all_ranks_captured"] = bool(int(ok.item()))
                if not graph_info.get("captured"):  # (rank 0 alone prints the line: say why here)
                    print(f"bench.py rank {rank}: no graph timing: {json.dumps(graph_info)}", file=sys.stderr, flush=True)
                if int(ok.item()) == 0 and graph_info.get("captured"):
                    graph_info.update(captured=False, note="another rank's capture failed: eager forwards timed")
        if graph_info and graph_info.get("captured"):
            # the timed steps replay the captured forward; the per-kernel HIP events and counters come
            # from the same number of eager steps right after (a replayed graph carries no host-side
            # per-launch events)
            fa._lib.fallback_stats(reset=True)  # (synchronises: outside the timed region)
            sync()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                replay()
            sync()
            if world > 1:
                dist.barrier()
            elapsed = time.perf_counter() - t0
            # the timed replays' own fallback counters (device-side: a replay counts them as an eager
            # forward does)
            graph_info["timed_replay_fallback"] = fa._lib.fallback_stats(reset=True)
            eager_elapsed, prof = instrumented(step)
            graph_info["eager_images_per_s"] = world * args.batch * args.steps / eager_elapsed
        else:
            elapsed, prof = instrumented(step)
            eager_elapsed = elapsed
    # how many launches / 64x64 output units of the timed steps left the fast path (a regression
    # there would otherwise be invisible in the line)
    fallback = fa._lib.fallback_stats() if cuda else None
    paths = {k: v for k, v in fa._lib.path_stats().items() if v} if cuda else None
    dense_fb = fa._lib.dense_stats() if cuda else None
    ktime = fa._lib.kernel_time(reset=True) if cuda else {}
    if args.dump_logits:  # one more step, after every counter was read (every rank: the gather is a collective)
        import numpy as np
        from fp8_quantization_amd.distributed import quantizers
        with torch.no_grad():
            local = model(x)
            final = gather_logits(local)
        if rank == 0:
            np.save(args.dump_logits, final.float().cpu().numpy())
        # (each rank: its own logits and FP8 state, for diagnosing a mismatch)
        st = {"logits": local.float().cpu().numpy()}
        for i, q in enumerate(quantizers(model)):
            st[f"q{i}_maxval"] = q.maxval.float().cpu().numpy()
            if isinstance(q.custom_bias, torch.Tensor):
                st[f"q{i}_bias"] = q.custom_bias.float().cpu().numpy()
        np.savez(f"{args.dump_logits}.rank{rank}.npz", **st)

    op_ms = sum(s.elapsed_time(e) for (s, e, _, _) in prof)
    op_macs = sum(m for (_, _, m, _) in prof)
    op_bytes = sum(b for (_, _, _, b) in prof)
    t = torch.tensor([elapsed, eager_elapsed], dtype=torch.float64, device=comm_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, eager_elapsed = float(t[0].item()), float(t[1].item())
    images = world * args.batch * args.steps

    if rank == 0:
        kernel, kdesc = dominant_kernel(args.expo_width, args.mant_width, args.v5_ofuf)
        launches = max(1, len(prof))
        avg_s = op_ms / 1e3 / launches
        op_achieved = 2.0 * (op_macs / launches) / avg_s / 1e12 if avg_s > 0 else None
        # the dominant kernel alone (fp8a_kernel_time: HIP events around each product-kernel launch,
        # on its stream, over the timed steps): its path's launches, time and approx-MACs
        kpath = {"gemm_f8mx_kernel": "f8mx", "gemm_tt16_kernel": "tt16", "gemm_tt_kernel": "tt",
                 "gemm_v5mx_kernel": "v5mx", "gemm_fast_kernel": "fast"}[kernel]
        kt = ktime.get(kpath, {})
        k_s = kt.get("ms", 0.0) / 1e3
        k_avg_s = k_s / kt["launches"] if kt.get("launches") else 0.0
        achieved = 2.0 * kt["macs"] / k_s / 1e12 if k_s > 0 else None
        pmc_name, pmc = pmc_summary(kernel, args.arch, args.expo_width, args.mant_width, args.batch)
        traffic = pmc.get("bytes_per_launch")
        # HBM: the PMC bytes per dispatch of the kernel x its timed dispatches / its timed time
        hbm_gbs = traffic * kt["dispatches"] / k_s / 1e9 if (traffic and k_s > 0) else None
        res = {
            "metric": metric_name(args.arch, args.expo_width, args.mant_width, args.v5_ofuf, args.no_approx),
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
                "workload": f"{arch_desc} E{args.expo_width}M{args.mant_width} "
                            + ("PTQ forward with approx_flag off (the exact product of the quantized operands, "
                               "original_quantize_res, " if args.no_approx else
                               "approx_v5 integer-adder forward (withComp, sim_hw_add_OFUF, with_OF_opt, with_UF_opt, "
                               if args.v5_ofuf else f"approx_v9 forward (dnsmp_factor=3, withComp={args.with_comp}, "
                               "with_s2nn2s_opt, quant_btw_mult_accu, ")
                            + ("zero error table (opt-in extension: the reference has none for this format), "
                               if (args.expo_width, args.mant_width) not in ((4, 3), (3, 4), (2, 5)) else "")
                            + "res_quantizer, fixed ranges), ImageNet-shaped synthetic batch, random-init weights"
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
                "kernel": f"{kernel} ({kdesc}); achieved / frac: the kernel alone (HIP events around its "
                          "launches); op_*: the whole approx op with its operand pre-decode, split-K reduce and "
                          "gated exact kernels",
                "achieved": achieved,
                "peak": FP32_VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / FP32_VALU_PEAK_TFLOPS if achieved else None,
                "kernel_frac": achieved / FP32_VALU_PEAK_TFLOPS if achieved else None,
                "kernel_avg_ms": k_avg_s * 1e3 if k_avg_s else None,
                "op_achieved": op_achieved,
                "op_frac": op_achieved / FP32_VALU_PEAK_TFLOPS if op_achieved else None,
                "op_avg_ms": avg_s * 1e3,
                "traffic": traffic,
                "hbm_gbs": hbm_gbs,
                "hbm_frac": hbm_gbs / HBM_PEAK_GBS if hbm_gbs else None,
                "valu_busy": pmc.get("valu_busy"),
                "valu_insts_per_simd_cycle": pmc.get("valu_instr_per_simd_cycle"),
                "wave_cycles": pmc.get("wave_cycles"),
                "pmc_summary": f"profiles/{pmc_name}" if pmc_name else None,
                "algorithmic": f"2 FLOP per approx-MAC; kernel: {kt.get('macs', 0) / max(1, kt.get('launches', 0)):.4g} "
                               f"approx-MAC per launch over {kt.get('launches', 0)} launches "
                               f"({kt.get('dispatches', 0)} dispatches), {k_avg_s * 1e3:.3f} ms avg launch; op: "
                               f"{op_macs / launches:.4g} approx-MAC per launch over {launches} launches, "
                               f"{avg_s * 1e3:.3f} ms avg (HIP events)",
                "hbm_note": "hbm_gbs = PMC HBM bytes per dispatch of the kernel (traffic, FETCH_SIZE x 2 + WRITE_SIZE, "
                            "tools/prof_summary.py) x its timed dispatches / its timed time; valu_busy = rocprof's "
                            "VALUBusy (4 x SQ_ACTIVE_INST_VALU / (SIMDs x GRBM_GUI_ACTIVE per XCD)), summed over "
                            "resident waves, so it counts a wave's cycles inside a VALU instruction, not VALU pipe "
                            "occupancy; wave_cycles: SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY shares",
                "approx_macs_per_s": op_macs / (op_ms / 1e3) if op_ms > 0 else None,
                # (op_ms comes from the eager instrumented steps: their share of those steps)
                "gemm_share_of_step": op_ms / 1e3 / eager_elapsed,
            },
        }
        if args.no_approx and cuda:
            gbs = op_bytes / (op_ms / 1e3) / 1e9 if op_ms > 0 else None
            # the dense GEMM kernel alone (fp8a_kernel_time's dense slot: HIP events around each
            # dn_gemm* launch; its MAC slot carries the launches' algorithmic bytes)
            dk = ktime.get("dense", {})
            dk_s = dk.get("ms", 0.0) / 1e3
            dk_gbs = dk["macs"] / dk_s / 1e9 if dk_s > 0 else None
            dpmc_name, dpmc = pmc_summary("dn_gemm_bf16", args.arch, args.expo_width, args.mant_width, args.batch,
                                          strict=True)
            dtraffic = dpmc.get("bytes_per_launch")
            dhbm = dtraffic * dk["dispatches"] / dk_s / 1e9 if (dtraffic and dk_s > 0) else None
            res["roofline"] = {
                "bound": "hbm",
                "kernel": "dn_gemm_bf16 (csrc/gemm_dense.h: the exact product on the bf16 matrix core, "
                          "implicit-GEMM conv / matmul, groups = 1) and dn_dw3_kernel (the depthwise convs, LDS-staged "
                          "fp32 FMAs); timed per op with its operand packing and gated fp32 units",
                "achieved": gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS if gbs else None,
                "traffic": dtraffic,
                "kernel_achieved": dk_gbs,
                "kernel_frac": dk_gbs / HBM_PEAK_GBS if dk_gbs else None,
                "kernel_avg_ms": dk_s * 1e3 / dk["launches"] if dk.get("launches") else None,
                "kernel_algorithmic_bytes_per_launch": dk["macs"] / dk["launches"] if dk.get("launches") else None,
                "hbm_gbs": dhbm,
                "hbm_frac": dhbm / HBM_PEAK_GBS if dhbm else None,
                "valu_busy": dpmc.get("valu_busy"),
                "wave_cycles": dpmc.get("wave_cycles"),
                "pmc_summary": f"profiles/{dpmc_name}" if dpmc_name else None,
                "algorithmic": f"fp32 operands read once + fp32 output written once: {op_bytes / launches:.4g} B per "
                               f"launch avg over {launches} launches, {avg_s * 1e3:.3f} ms avg launch (HIP events); "
                               f"{2.0 * op_macs / (op_ms / 1e3) / 1e12 if op_ms > 0 else 0:.1f} TFLOP/s of exact "
                               f"products (fp8 MFMA dense peak {FP8_MFMA_PEAK_TFLOPS:.0f})",
                "gemm_share_of_step": op_ms / 1e3 / eager_elapsed,
            }
            res["dense_fp32_units"] = dict(dense_fb, note="timed steps only: dense launches with 64x64 units "
                                                          "recomputed in fp32 (blocks not exact in e4m3 / e5m2)")
        if graph_info is not None:
            res["hip_graph"] = graph_info
        if fallback is not None and not args.no_approx:
            res["fallback"] = dict(fallback, approx_launches=len(prof),
                                   note="timed steps only: exact_launches = launches whose gated exact kernel "
                                        "recomputed exact_units 64x64 output units; f32_reruns = E3M4 launches "
                                        "rerun in the f32 tile-table form; tb_launches = depthwise launches "
                                        "recomputed by the literal restatement")
        if paths is not None:
            res["gemm_paths"] = dict(paths, note="timed steps only: approx GEMM launches per kernel path "
                                                 "(fp8a_path_stats)")
        if world == 1 and not args.no_cpu_baseline and (args.expo_width, args.mant_width) == (4, 3) \
                and not args.no_approx:
            res["cpu_baseline"] = cpu_baseline(shapes, get_error_table_NN(4, 3, args.with_comp, 3), args.cpu_columns)
            res["speedup_vs_cpu_baseline"] = res["value"] / res["cpu_baseline"]["value"]
        if not cuda:
            res.pop("roofline")
        return res
    return None


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(local_rank, world, port, argv, worker_init):
    """One rank of a `--gpus N` launch: the environment torch.distributed.run would give it,
    then the same entry point."""
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if worker_init is not None:
        worker_init()
    main(argv)


def launch(args, argv, worker_init=None):
    """`--gpus N` without a launcher: start N fresh rank processes (spawn) from this process,
    which has not touched the GPU (it only parsed arguments), and wait for them.  Rank 0 prints
    the line.  `worker_init` (a picklable top-level function) runs first in every rank: the CPU
    rehearsal's stand-ins (tests/test_distributed_cpu.py)."""
    import torch.multiprocessing as mp
    mp.start_processes(_spawned, args=(args.gpus, _free_port(), argv, worker_init), nprocs=args.gpus,
                       join=True, start_method="spawn")


def main(argv=None, worker_init=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args, argv, worker_init)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; reporting {world} GPUs", file=sys.stderr)
    if args.device == "cpu":  # the gloo rehearsal (tests): same control flow, no GPU
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        if args.share_device and args.dist_backend != "gloo":
            raise SystemExit("bench.py: --share-device needs --dist-backend gloo (RCCL wants one GPU per rank)")
        dev = torch.device("cuda", 0 if args.share_device else local)
        if world > 1:
            torch.cuda.set_device(dev)
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group("gloo", rank=rank, world_size=world)
    if world > 1:
        world = dist.get_world_size()
    res = run(args, dev, rank, world)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
