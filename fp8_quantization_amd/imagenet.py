"""ImageNet validation of an approx-FP8 model: the reference's `validate-quantized` protocol on
one or many GPUs.

    python -m fp8_quantization_amd.imagenet --images-dir /data/imagenet --arch resnet18 \
        [--weights resnet18.pth] [--mini-test] [--batch-size 64]
    python -m torch.distributed.run --nproc-per-node 8 -m fp8_quantization_amd.imagenet ...

Restates image_net.py:59-202 of the reference without click / ignite / torchvision:
  * data: <images-dir>/val/<integer class>/<image> folders, labels = the folder's integer
    (imagenet_dataloaders.py:105-139), val transform Resize(image_size + 24) -> CenterCrop ->
    ToTensor -> Normalize(ImageNet mean / std) (:67-84) done with PIL + torch;
  * calibration: estimate_ranges, `--num-est-batches` batches (default 1, the reference's
    num_est_batches) of <images-dir>/train (or of val when no train split is present),
    set_quant_state, fix_ranges (image_net.py:76-91, quantization/utils.py:74-115);
  * evaluation: the reference's "mini_test" (CustomBatchSampler num_batches=10, start_index=5,
    step=300 over the val loader, image_net.py:172-179) or the full val set; top-1, top-5 and
    cross-entropy loss;
  * multi-GPU: one process per GPU; rank 0 calibrates, its FP8 ranges are broadcast, the
    evaluated batches are sharded over ranks and the logits all-gathered (RCCL) for scoring.
BN re-estimation (a QAT utility that needs the train split) is not run: the reference's
`--no-reestimate-bn-stats` protocol.
Without a dataset (`--synthetic N`), random images / labels exercise the same path.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
_EXTS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def resize_shorter(img, size):
    """torchvision Resize(int) on a PIL image: the shorter side becomes `size` (bilinear)."""
    from PIL import Image
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    if short == size:
        return img
    new_short, new_long = size, int(size * long / short)
    new_w, new_h = (new_short, new_long) if w <= h else (new_long, new_short)
    return img.resize((new_w, new_h), Image.BILINEAR)


def center_crop(img, size):
    """torchvision CenterCrop: top = round((h - size) / 2), left = round((w - size) / 2)."""
    w, h = img.size
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return img.crop((left, top, left + size, top + size))


def val_transform(img, image_size=224):
    img = center_crop(resize_shorter(img.convert("RGB"), image_size + 24), image_size)
    x = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).float().div_(255.0)
    mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(3, 1, 1)
    return (x - mean) / std


class NumericImageFolder(torch.utils.data.Dataset):
    """ImageFolder whose class directories are integers and whose labels are those integers
    (imagenet_dataloaders.py:105-133); samples ordered like ImageFolder (class dirs sorted by
    name, files sorted)."""

    def __init__(self, root, image_size=224):
        self.root, self.image_size = root, image_size
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        try:
            labels = {c: int(c) for c in classes}
        except ValueError:
            raise ValueError("all class directory names must be integers, e.g. '0', '1', '2', ...")
        self.samples = []
        for c in classes:
            for dirpath, _, files in sorted(os.walk(os.path.join(root, c))):
                for f in sorted(files):
                    if f.lower().endswith(_EXTS):
                        self.samples.append((os.path.join(dirpath, f), labels[c]))

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        from PIL import Image
        path, label = self.samples[i]
        with open(path, "rb") as f:
            img = Image.open(f)
            img.load()
        return val_transform(img, self.image_size), label


class SyntheticImages(torch.utils.data.Dataset):
    def __init__(self, n, image_size=224, classes=1000, seed=0):
        self.n, self.image_size, self.classes, self.seed = n, image_size, classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        return torch.randn((3, self.image_size, self.image_size), generator=g), int(
            torch.randint(self.classes, (1,), generator=g))


def mini_test_batches(n_batches_total, num_batches=10, start_index=5, step=300):
    """Batch indices CustomBatchSampler visits in sequential mode (CustomBatchSampler.py:20-29)."""
    out = []
    for i in range(n_batches_total):
        if i < start_index:
            continue
        if (i - start_index) % step == 0:
            out.append(i)
            if (i - start_index) // step + 1 >= num_batches:
                break
    return out


def build_model(arch, weights, cfg, image_size=224):
    from . import resnet_workload as rw
    if arch == "resnet18":
        return rw.resnet18_approx(weights=weights, **cfg)
    if arch == "resnet50":
        return rw.resnet50_approx(weights=weights, **cfg)
    if arch == "mobilenet_v2":
        from .mobilenet_workload import MobileNetV2, QuantizedMobileNetV2
        fp = MobileNetV2(input_size=image_size)  # its head pools with AvgPool2d(input_size // 32)
        if weights:
            sd = torch.load(weights, map_location="cpu", weights_only=True)
            fp.load_state_dict(sd.get("state_dict", sd))
        return QuantizedMobileNetV2(fp, input_size=(1, 3, image_size, image_size), **rw.approx_qparams(**cfg))
    if arch == "vit_b16":  # models/vit_quantized_approx.py (the registry's vit_quantized_approx)
        from .vit_workload import vit_b16_approx
        return vit_b16_approx(weights=weights, image_size=image_size, **cfg)
    raise ValueError(f"unknown architecture {arch}")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--images-dir", default=None)
    ap.add_argument("--synthetic", type=int, default=0, help="N random images instead of a dataset")
    ap.add_argument("--arch", default="resnet18", choices=["resnet18", "resnet50", "mobilenet_v2", "vit_b16"])
    ap.add_argument("--weights", default=None, help="float (torchvision-format) state dict")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--batch-size", type=int, default=16)
    ap.add_argument("--num-workers", type=int, default=8)
    ap.add_argument("--num-est-batches", type=int, default=1)
    ap.add_argument("--mini-test", action="store_true", help="the reference's 10-batch evaluation")
    ap.add_argument("--max-batches", type=int, default=0, help="cap on evaluated batches (0 = all)")
    ap.add_argument("--expo-width", type=int, default=4)
    ap.add_argument("--mant-width", type=int, default=3)
    ap.add_argument("--dnsmp-factor", type=int, default=3)
    ap.add_argument("--with-comp", action="store_true")
    ap.add_argument("--no-approx", action="store_true", help="approx_flag off (quantized, exact products)")
    ap.add_argument("--no-s2n", action="store_true")
    ap.add_argument("--no-qbma", action="store_true")
    ap.add_argument("--output", default=None, help="also write the result JSON here")
    return ap.parse_args(argv)


def _loader(ds, batch, workers, indices=None):
    if indices is not None:
        ds = torch.utils.data.Subset(ds, indices)
    return torch.utils.data.DataLoader(ds, batch_size=batch, shuffle=False, num_workers=workers, pin_memory=True)


def validate(model, val, train, args, dev, rank=0, ws=1, source=""):
    """Calibrate on rank 0 (ranges broadcast), evaluate the (mini_test or full) batches sharded
    over ranks with one packed all-gather per step; rank 0 returns the result dict (None on
    the other ranks).  `model` is already on `dev` in eval mode."""
    from .distributed import calibrate_on_rank0, gather_scored, score

    def cal_batches():
        for i, (x, _) in enumerate(_loader(train, args.batch_size, args.num_workers)):
            yield x.to(dev, non_blocking=True)
            if i >= args.num_est_batches - 1:
                break
    calibrate_on_rank0(model, cal_batches())

    # evaluated batches (mini_test or all), sharded over ranks; each global step every rank
    # runs one batch (or none) and the packed logits / labels are all-gathered once
    nb = (len(val) + args.batch_size - 1) // args.batch_size
    batches = mini_test_batches(nb) if args.mini_test else list(range(nb))
    if args.max_batches:
        batches = batches[:args.max_batches]
    mine = batches[rank::ws]
    steps = (len(batches) + ws - 1) // ws
    n_cls = [m for m in model.modules() if hasattr(m, "out_features")][-1].out_features
    idx = [i for b in mine for i in range(b * args.batch_size, min(len(val), (b + 1) * args.batch_size))]
    it = iter(_loader(val, args.batch_size, args.num_workers, idx)) if idx else iter(())
    correct1 = correct5 = seen = 0
    loss_sum = 0.0
    t0 = time.perf_counter()
    with torch.inference_mode():
        for s in range(steps):
            if s < len(mine):
                x, y = next(it)
                logits = model(x.to(dev, non_blocking=True))
                y = y.to(dev)
            else:  # this rank has no batch left this step: it contributes no valid rows
                logits = torch.zeros((0, n_cls), device=dev)
                y = torch.zeros(0, dtype=torch.long, device=dev)
            L, Y = gather_scored(logits, y, args.batch_size)
            if rank == 0 and Y.numel():
                hits, loss = score(L, Y)
                correct1 += hits[1]
                correct5 += hits[5]
                loss_sum += loss
                seen += int(Y.numel())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if rank != 0:
        return None
    return dict(arch=args.arch, data=source, images=seen, top_1_accuracy=correct1 / max(1, seen),
                top_5_accuracy=correct5 / max(1, seen), loss=loss_sum / max(1, seen), images_per_s=seen / elapsed,
                n_gpus=ws, evaluate_param="mini_test" if args.mini_test else "full_test")


def datasets(args):
    if args.synthetic:
        val = SyntheticImages(args.synthetic, args.image_size)
        train = SyntheticImages(args.batch_size * args.num_est_batches, args.image_size, seed=1)
        return val, train, f"synthetic ({args.synthetic} random images)"
    val = NumericImageFolder(os.path.join(args.images_dir, "val"), args.image_size)
    tdir = os.path.join(args.images_dir, "train")
    train = NumericImageFolder(tdir, args.image_size) if os.path.isdir(tdir) else val
    return val, train, args.images_dir + ("" if train is not val else " (calibrated on val: no train split)")


def approx_cfg(args):
    cfg = dict(expo_width=args.expo_width, mant_width=args.mant_width, dnsmp_factor=args.dnsmp_factor,
               withComp=args.with_comp, with_approx=True, with_s2nn2s_opt=not args.no_s2n,
               quant_btw_mult_accu=not args.no_qbma)
    if args.no_approx:
        # the reference's canonical no-approx run (scripts/image_net.sh:42-45): exact product, then
        # the res quantizer through the original_quantize_res branch
        cfg["run_method"] = dict(approx_flag=False, quantize_after_mult_and_add=False, res_quantizer_flag=True,
                                 original_quantize_res=True)
    return cfg


def main(argv=None):
    args = parse(argv)
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("the approx path needs a HIP device")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        dist.init_process_group("nccl", device_id=dev)
    val, train, source = datasets(args)
    cfg = approx_cfg(args)
    model = build_model(args.arch, args.weights, cfg, args.image_size).to(dev).eval()
    res = validate(model, val, train, args, dev, rank, ws, source)
    if rank == 0:
        res["approx_params"] = cfg
        print(json.dumps(res), flush=True)
        if args.output:
            with open(args.output, "w") as f:
                json.dump(res, f, indent=1)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
