"""Multi-GPU plumbing of the approx validation path.

Inference images are independent, so the validation set is sharded contiguously over ranks
(one process per GPU) with no collective in the data path.  The collectives:
  * once, before the data path: rank 0's float model state (parameters and buffers: the BN
    statistics of a synthetic-weights model are estimated per process) and, after rank 0 alone
    has calibrated, its FP8 ranges (every FPQuantizer.maxval / sign_bits, a few KB) are
    broadcast, so all ranks use identical weights and bA / bB / bR (calibrate_on_rank0);
  * per validation batch: ONE all-gather (RCCL over xGMI on MI355X; gloo on CPU) of a packed
    [B, classes + 2] float tensor -- the logits, the label and a valid-row flag per row
    (gather_scored) -- from which rank 0 scores top-1 / top-5 / loss.  The benchmark step
    gathers the logits alone (gather_logits).
"""
import torch
import torch.distributed as dist
import torch.nn.functional as F


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


def comm_device():
    """The device a collective's tensors must live on: the current GPU for RCCL ("nccl"), the
    host for gloo."""
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_model_state(model, src=0):
    """Every parameter and buffer of `model` from rank `src` (identical architecture on every
    rank, so shapes agree): ONE broadcast per dtype of the flattened tensors, on the
    collective's device, copied back in place."""
    ws, _ = world()
    if ws == 1:
        return
    dev = comm_device()
    groups = {}
    for t in list(model.parameters()) + list(model.buffers()):
        groups.setdefault(t.dtype, []).append(t)
    with torch.no_grad():
        for dtype, ts in groups.items():
            wire = torch.uint8 if dtype == torch.bool else dtype
            flat = torch.cat([t.detach().reshape(-1).to(device=dev, dtype=wire) for t in ts])
            dist.broadcast(flat, src)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view(t.shape).to(dtype))
                off += n


_HDR = 16  # per quantizer: maxval numel, sign_bits, ndim, 5 dims; custom_bias numel (-1: None), ndim, 5 dims


def broadcast_quant_state(model, src=0):
    """Make every rank's FP8 ranges identical to rank `src`'s with two broadcasts in all: one
    int64 header [quantizers, 16] (maxval element count, sign_bits and shape; custom_bias element
    count and shape) and one float32 buffer of every quantizer's maxval and custom_bias.  Ranks that
    never calibrated receive the calibrated (e.g. per-channel) shapes.

    custom_bias travels too: an activation / weight quantizer rewrites it on every forward, but the
    res quantizer of a fixed-range approx layer runs only during calibration (hijacker.py:77-115),
    so its custom_bias -- the layer's bR -- exists only where calibration ran; without it the other
    ranks would fall back to 2^(E-1) (approx_calculation.py:766-767) and compute other products.

    Both tensors are built on the collective's device (RCCL rejects host tensors; a quantizer that
    never ran a forward still holds its maxval on the host), and each received tensor is moved to
    the model's device -- the GPU the forward runs on (the collective's own device under RCCL; gloo
    on a GPU model stages through the host)."""
    ws, rank = world()
    if ws == 1:
        return
    qs = quantizers(model)
    if not qs:
        return
    dev = comm_device()
    hdr = torch.zeros((len(qs), _HDR), dtype=torch.int64)
    if rank == src:
        for i, q in enumerate(qs):
            shp = list(q.maxval.shape)
            cb = q.custom_bias
            cshp = list(cb.shape) if isinstance(cb, torch.Tensor) else []
            if len(shp) > 5 or len(cshp) > 5:
                raise ValueError(f"maxval / custom_bias of rank {rank} have more than 5 dims")
            hdr[i, :3 + len(shp)] = torch.tensor([q.maxval.numel(), int(q.sign_bits), len(shp)] + shp)
            hdr[i, 8:10 + len(cshp)] = torch.tensor([cb.numel() if isinstance(cb, torch.Tensor) else -1, len(cshp)]
                                                    + cshp)
    hdr = hdr.to(dev)
    dist.broadcast(hdr, src)
    hdr = hdr.cpu()
    total = int(hdr[:, 0].sum() + hdr[:, 8].clamp(min=0).sum())
    if rank == src:
        parts = []
        for q in qs:
            parts.append(q.maxval.detach().reshape(-1).to(device=dev, dtype=torch.float32))
            if isinstance(q.custom_bias, torch.Tensor):
                parts.append(q.custom_bias.detach().reshape(-1).to(device=dev, dtype=torch.float32))
        flat = torch.cat(parts)
    else:
        flat = torch.empty(total, dtype=torch.float32, device=dev)
    dist.broadcast(flat, src)
    # the ranges live where the model runs (gloo's host buffers are staging only)
    p0 = next(iter(model.parameters()), None)
    flat = flat.to(p0.device if p0 is not None else dev)
    off = 0
    for q, h in zip(qs, hdr.tolist()):
        n, sb, nd = h[0], h[1], h[2]
        q.maxval = flat[off:off + n].clone().view(h[3:3 + nd])
        q.sign_bits = sb
        off += n
        cn, cnd = h[8], h[9]
        if cn >= 0:
            cb = flat[off:off + cn].clone().view(h[10:10 + cnd])
            if rank != src:
                q.custom_bias = cb
                cb._fp8a_i32 = cb.reshape(-1).to(torch.int32)  # (as fp8_fake_quantize leaves it)
            off += cn


def calibrate_on_rank0(model, batches, src=0, quantized=False):
    """The reference's calibration (image_net.py:76-91: estimate_ranges, forward the
    calibration batches, fix_ranges) run by rank `src` alone; every other rank takes rank
    `src`'s model state and FP8 ranges by broadcast.  `batches` is an iterable of input
    tensors (only consumed on rank `src`).  quantized=True calls model.quantized() first (the
    benchmark's order), else set_quant_state(True, True) around the pass (the validate
    driver's)."""
    _, rank = world()
    broadcast_model_state(model, src)
    if quantized:
        model.quantized()
    model.estimate_ranges()
    if not quantized:
        model.set_quant_state(True, True)
    if rank == src:
        with torch.no_grad():
            for x in batches:
                model(x)
    if not quantized:
        model.set_quant_state(True, True)
    model.fix_ranges()
    broadcast_quant_state(model, src)


def gather_logits(logits):
    """All-gather equal-sized per-rank logits into [world * B, C] (rank order), returned on the
    logits' device.  RCCL gathers in place on the GPU; gloo (the one-GPU rehearsal of N ranks,
    bench.py --dist-backend gloo) stages GPU logits through the host."""
    ws, _ = world()
    if ws == 1:
        return logits
    dev = comm_device()
    src = logits.contiguous().to(dev)
    out = torch.empty((ws * logits.shape[0],) + tuple(logits.shape[1:]), dtype=logits.dtype, device=dev)
    dist.all_gather_into_tensor(out, src)
    return out.to(logits.device)


def gather_scored(logits, labels, batch):
    """One all-gather per validation step: this rank's logits [n, C] (n <= batch; n = 0 for a
    rank without a batch this step), its labels [n], padded to `batch` rows and packed with a
    label column and a valid-row flag into float32 [batch, C + 2] (class indices < 2^24 are
    exact).  Returns the valid rows of every rank in rank order: (logits [N, C], labels [N])."""
    n, C = logits.shape
    packed = torch.zeros((batch, C + 2), dtype=torch.float32, device=logits.device)
    packed[:n, :C] = logits.float()
    packed[:n, C] = labels.float()
    packed[:n, C + 1] = 1.0
    allp = gather_logits(packed)
    valid = allp[:, C + 1] > 0
    return allp[valid, :C], allp[valid, C].long()


def score(logits, labels, ks=(1, 5)):
    """(top-k hit counts, summed cross-entropy) of a scored batch."""
    top = logits.topk(max(ks), dim=1).indices
    hit = top.eq(labels.view(-1, 1))
    return ({k: int(hit[:, :k].any(dim=1).sum().item()) for k in ks},
            float(F.cross_entropy(logits, labels, reduction="sum")) if labels.numel() else 0.0)


def topk_correct(logits, labels, ks=(1, 5)):
    return score(logits, labels, ks)[0]
