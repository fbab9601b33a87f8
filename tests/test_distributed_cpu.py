"""World-size-2 gloo rehearsal of the sharded validation path (fp8_quantization_amd.distributed).

The approx kernels need a GPU, so the per-rank model here is a plain torch stand-in; what is
under test is the sharding, the one-time quantizer-state broadcast and the logits all-gather.
"""
import os
import socket

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
        broadcast_quant_state(holder, src=0)
        q.put((rank, allg, topk_correct(allg, labels), float(holder.q.maxval[0]), (x @ w)))
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
    for rank, allg, acc, mx, _ in res:
        assert torch.equal(allg, full)          # gathered logits == unsharded logits
        assert mx == 1.0                        # rank 0's ranges everywhere
        assert acc == res[0][2]
