"""Multi-GPU plumbing of the approx validation path.

Inference images are independent, so the validation set is sharded contiguously over ranks
(one process per GPU) with no collective in the data path.  Exactly two collectives exist:
  * broadcast_quant_state: rank 0's calibrated FP8 ranges (every FPQuantizer.maxval, a few KB)
    go to every rank once, so all ranks use identical bA / bB / bR;
  * gather_logits: one all-gather of the [B, classes] logits per validation batch (RCCL over
    xGMI on MI355X; gloo on CPU), from which rank 0 scores top-1 / top-5.
"""
import torch
import torch.distributed as dist


def world():
    return (dist.get_world_size(), dist.get_rank()) if dist.is_available() and dist.is_initialized() else (1, 0)


def shard_range(n, rank, world_size):
    """Contiguous [lo, hi) slice of n items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def quantizers(model):
    from .quantization.fp8_quantizer import FPQuantizer
    return [m for m in model.modules() if isinstance(m, FPQuantizer)]


def broadcast_quant_state(model, src=0):
    """Make every rank's FP8 ranges identical to rank `src`'s (one broadcast per quantizer)."""
    ws, _ = world()
    if ws == 1:
        return
    for q in quantizers(model):
        mx = q.maxval.detach().clone().contiguous()
        n = torch.tensor([mx.numel()], dtype=torch.int64, device=mx.device)
        dist.broadcast(n, src)
        if mx.numel() != int(n.item()):
            mx = torch.empty(int(n.item()), dtype=mx.dtype, device=mx.device)
        dist.broadcast(mx, src)
        q.maxval = mx
        q.sign_bits = int(q.sign_bits)


def gather_logits(logits):
    """All-gather equal-sized per-rank logits into [world * B, C] (rank order)."""
    ws, _ = world()
    if ws == 1:
        return logits
    out = torch.empty((ws * logits.shape[0],) + tuple(logits.shape[1:]), dtype=logits.dtype, device=logits.device)
    dist.all_gather_into_tensor(out, logits.contiguous())
    return out


def topk_correct(logits, labels, ks=(1, 5)):
    top = logits.topk(max(ks), dim=1).indices
    hit = top.eq(labels.view(-1, 1))
    return {k: int(hit[:, :k].any(dim=1).sum().item()) for k in ks}
