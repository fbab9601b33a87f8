"""World-size-2 gloo rehearsal of the sharded validation path (fp8_quantization_amd.distributed).

The approx kernels need a GPU, so the per-rank model here is a plain torch stand-in; what is
under test is the sharding, the one-time quantizer-state broadcast and the logits all-gather.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fp8_quantization_amd.distributed import gather_logits, shard_range, topk_correct


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from fp8_quantization_amd.distributed import broadcast_quant_state
        from fp8_quantization_amd.quantization.fp8_quantizer import FPQuantizer
        torch.manual_seed(0)
        n, d, c = 10, 6, 7
        x = torch.randn(n, d)
        labels = torch.randint(0, c, (n,))
        w = torch.randn(d, c)
        lo, hi = shard_range(n, rank, ws)
        logits = x[lo:hi] @ w
        allg = gather_logits(logits)
        # calibrated ranges differ per rank before the broadcast, agree after
        holder = torch.nn.Module()
        holder.q = FPQuantizer(n_bits=8, mantissa_bits=3, set_maxval=True)
        holder.q.maxval = torch.tensor([1.0 + rank])
        # a res quantizer's custom_bias (bR) exists only where calibration ran: it must travel too
        holder.q.custom_bias = torch.tensor([5.0]) if rank == 0 else None
        # a per-channel quantizer: rank 0 calibrated it ([3, 1] ranges, unsigned); the other rank
        # never ran a forward and holds its maxval on a device the collective cannot use (here
        # 'meta', on a GPU box the host while RCCL needs the GPU) -- it must not be touched
        holder.w = FPQuantizer(n_bits=8, mantissa_bits=3, set_maxval=True)
        if rank == 0:
            holder.w.maxval = torch.tensor([[0.5], [2.0], [8.0]])
            holder.w.sign_bits = 0
        else:
            holder.w.maxval = torch.empty(1, device="meta")
        broadcast_quant_state(holder, src=0)
        # model state: one flattened broadcast per dtype (float parameters, int64 / bool buffers)
        from fp8_quantization_amd.distributed import broadcast_model_state
        m = torch.nn.Linear(3, 2)
        with torch.no_grad():
            m.weight.fill_(float(rank))
        m.register_buffer("count", torch.tensor([7 * (rank + 1)], dtype=torch.int64))
        m.register_buffer("mask", torch.tensor([rank == 0, rank == 1]))
        broadcast_model_state(m, src=0)
        state = dict(w=m.weight.tolist(), count=m.count.tolist(), mask=m.mask.tolist(), wdev=str(holder.w.maxval.device),
                     wmax=holder.w.maxval.tolist(), wsign=holder.w.sign_bits,
                     qcb=holder.q.custom_bias.tolist(), qcb_i32=holder.q.custom_bias._fp8a_i32.tolist()
                     if rank else [5], wcb=holder.w.custom_bias)
        # (tensors by value: a shared-memory handle can outlive this process and fail to open)
        q.put((rank, allg.numpy().copy(), topk_correct(allg, labels), float(holder.q.maxval[0]), (x @ w).numpy().copy(),
               state))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_everything():
    for n in (0, 1, 7, 256, 1001):
        for ws in (1, 2, 3, 8):
            parts = [shard_range(n, r, ws) for r in range(ws)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


def test_gloo_world2_gather_and_broadcast():
    ws = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    full = res[0][4]
    for rank, allg, acc, mx, _, st in res:
        assert np.array_equal(allg, full)       # gathered logits == unsharded logits
        assert mx == 1.0                        # rank 0's ranges everywhere
        assert acc == res[0][2]
        assert st["wdev"] == "cpu" and st["wmax"] == [[0.5], [2.0], [8.0]] and st["wsign"] == 0
        assert st["w"] == [[0.0] * 3] * 2 and st["count"] == [7] and st["mask"] == [True, False]
        assert st["qcb"] == [5.0] and st["qcb_i32"] == [5] and st["wcb"] is None


# ---------------------------------------------------------------------------------------------
# The real control flow (imagenet.validate / bench.run) at world size 2 on gloo.  The approx
# ops need a GPU, so the conv / linear products run as torch stand-ins and the FP8 fake
# quantizer as the CPU oracle's restatement; the fused-launch paths are switched off (they have
# no stand-in).  Under test: rank-0-only calibration + state broadcast, batch sharding, the one
# packed all-gather per step and rank 0's scoring.
def _install_standins():
    import numpy as np
    import torch.nn.functional as F

    from fp8_quantization_amd import approx_calculation as ac
    from fp8_quantization_amd import model_wrap
    from fp8_quantization_amd.quantization import fp8_quantizer as fq
    from fp8_quantization_amd.quantization.hijacker import QuantizationHijacker
    from fp8_quantization_amd.quantization.quantized_folded_bn import BNFusedHijacker
    from oracle import oracle

    def fake_quant(x, maxval, n_bits, M, sign_bits=1, per_row=False):
        assert sign_bits == 1
        mx = torch.as_tensor(maxval, dtype=torch.float32).reshape(-1).cpu().numpy()
        out, bias = oracle.fp8_fake_quant(x.detach().cpu().numpy(), mx, n_bits - 1 - M, M, per_row and mx.size > 1)
        b = torch.from_numpy(np.ascontiguousarray(bias))
        if per_row and mx.size > 1:
            b = b.view([-1] + [1] * (x.dim() - 1))
        return torch.from_numpy(out).to(x.device), b

    fq.fp8_fake_quantize = fake_quant
    ac.approx_conv2d = lambda x, w, E, M, bA, bW, bR, table=None, flags=None, stride=(1, 1), padding=(0, 0), \
        dilation=(1, 1), groups=1, epilogue=None, qin=None, post=None: F.conv2d(x, w, None, stride, padding, dilation,
                                                                               groups)
    ac.approx_matmul = lambda A, B, E, M, bA, bB, bR, table=None, flags=None: A @ B
    QuantizationHijacker.fuse_input_quant = False
    BNFusedHijacker.fuse_bn_act = False
    ac.ApproxLinearMixin.fuse_linear_block = False
    model_wrap.FUSE_BLOCK = False


_VAL_ARGS = ["--synthetic", "10", "--batch-size", "4", "--num-workers", "0", "--arch", "mobilenet_v2",
             "--image-size", "32"]


def _validate_once(rank, ws):
    from fp8_quantization_amd import imagenet
    args = imagenet.parse(_VAL_ARGS)
    val, train, source = imagenet.datasets(args)
    torch.manual_seed(100 + rank)  # different init per rank: the state broadcast must fix it
    model = imagenet.build_model(args.arch, None, imagenet.approx_cfg(args), args.image_size).eval()
    res = imagenet.validate(model, val, train, args, torch.device("cpu"), rank, ws, source)
    from fp8_quantization_amd.distributed import quantizers
    return res, [q.maxval.reshape(-1).tolist() for q in quantizers(model)]  # plain lists: cross the queue safely


def _flow_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        _install_standins()
        res, mx = _validate_once(rank, ws)
        res = json.loads(json.dumps(res)) if res is not None else None
        import bench
        bres = bench.run(bench.parse(["--arch", "mobilenet_v2", "--batch", "2", "--steps", "1", "--warmup", "1",
                                      "--cal-batch", "2", "--bn-stats-batches", "0", "--no-cpu-baseline"]),
                         torch.device("cpu"), rank, ws)
        q.put((rank, res, mx, json.loads(json.dumps(bres)) if bres is not None else None))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None, None))
        raise
    finally:
        dist.destroy_process_group()


def _single_worker(q):
    torch.set_num_threads(1)
    _install_standins()  # (in a child process: the stand-ins never leak into this test session)
    res, _ = _validate_once(0, 1)
    q.put(json.loads(json.dumps(res)))


def test_gloo_world2_validate_and_bench_flow():
    ws = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_flow_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(ws)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, r, m, _ in res:
        assert m is not None, r  # a worker failed: its traceback
    (_, r0, mx0, b0), (_, r1, mx1, b1) = res
    assert r1 is None and b1 is None                      # only rank 0 scores / reports
    assert len(mx0) == len(mx1) and mx0 == mx1  # rank 0's ranges everywhere
    # the same validation unsharded (world size 1, rank 0's initialisation)
    p1 = ctx.Process(target=_single_worker, args=(q,))
    p1.start()
    single = q.get(timeout=600)
    p1.join(timeout=60)
    assert r0["images"] == single["images"] == 10
    assert r0["top_1_accuracy"] == single["top_1_accuracy"] and r0["top_5_accuracy"] == single["top_5_accuracy"]
    assert abs(r0["loss"] - single["loss"]) <= 1e-5 * abs(single["loss"])
    assert b0["n_gpus"] == 2 and b0["config"]["global_batch"] == 4 and b0["value"] > 0


def test_bench_main_gpus2_spawns_ranks(capfd):
    """`bench.py --gpus 2` with no launcher environment starts the two ranks itself (spawned
    from a parent that touches no GPU) and rank 0 reports n_gpus = 2 -- the driver's scaling
    command form (here on the CPU rehearsal device: gloo and torch stand-ins)."""
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        assert k not in os.environ
    bench.main(["--gpus", "2", "--device", "cpu", "--arch", "mobilenet_v2", "--batch", "2", "--steps", "1",
                "--warmup", "1", "--cal-batch", "2", "--bn-stats-batches", "0", "--no-cpu-baseline"],
               worker_init=_install_standins)
    lines = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, lines  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 4 and line["config"]["parallelism"] == "dp2"
    assert line["value"] > 0
