"""Host-side pieces of the ImageNet validate driver (fp8_quantization_amd/imagenet.py)."""
import os

import numpy as np
import pytest
import torch

from fp8_quantization_amd import imagenet as inet


def _png(path, w, h, seed):
    from PIL import Image
    rng = np.random.default_rng(seed)
    Image.fromarray(rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)).save(path)


def test_resize_and_center_crop_follow_torchvision_rules():
    from PIL import Image
    img = Image.new("RGB", (500, 375))
    r = inet.resize_shorter(img, 248)
    assert r.size == (int(248 * 500 / 375), 248)          # shorter side -> 248, long side floored
    c = inet.center_crop(r, 224)
    assert c.size == (224, 224)
    tall = inet.resize_shorter(Image.new("RGB", (300, 640)), 248)
    assert tall.size == (248, int(248 * 640 / 300))


def test_val_transform_normalises():
    from PIL import Image
    img = Image.new("RGB", (256, 256), color=(124, 116, 104))   # ~ the ImageNet mean
    x = inet.val_transform(img, 224)
    assert x.shape == (3, 224, 224) and x.dtype == torch.float32
    assert float(x.abs().max()) < 0.01


def test_numeric_folder_labels_are_folder_integers(tmp_path):
    root = tmp_path / "val"
    for cls, n in (("10", 2), ("2", 1), ("7", 3)):
        os.makedirs(root / cls)
        for i in range(n):
            _png(root / cls / f"img{i}.png", 40 + i, 30, hash((cls, i)) % 1000)
    ds = inet.NumericImageFolder(str(root), image_size=16)
    assert len(ds) == 6
    # ImageFolder order: class directories sorted by name ("10" < "2" < "7"), labels = int(name)
    assert [lbl for _, lbl in ds.samples] == [10, 10, 2, 7, 7, 7]
    x, y = ds[3]
    assert x.shape == (3, 16, 16) and y == 7


def test_numeric_folder_rejects_non_integer_classes(tmp_path):
    os.makedirs(tmp_path / "val" / "n01440764")
    with pytest.raises(ValueError):
        inet.NumericImageFolder(str(tmp_path / "val"))


def test_mini_test_batches_match_custom_batch_sampler():
    # CustomBatchSampler(num_batches=10, start_index=5, step=300) over ImageNet val at batch 16
    assert inet.mini_test_batches(3125) == [5 + 300 * i for i in range(10)]
    assert inet.mini_test_batches(700) == [5, 305, 605]
    assert inet.mini_test_batches(3) == []


def test_synthetic_images_are_deterministic():
    a, b = inet.SyntheticImages(4, 8), inet.SyntheticImages(4, 8)
    xa, ya = a[2]
    xb, yb = b[2]
    assert torch.equal(xa, xb) and ya == yb


def test_build_model_knows_every_bench_architecture():
    """The validate driver builds the same wrappers as bench.py (ViT-B/16 included)."""
    from fp8_quantization_amd.approx_calculation import QCustomLinearTorch
    from fp8_quantization_amd.imagenet import build_model
    from fp8_quantization_amd.vit_workload import QuantizedVisionTransformerForImageClassification
    cfg = dict(expo_width=4, mant_width=3, dnsmp_factor=3, withComp=False)
    m = build_model("vit_b16", None, cfg)
    assert isinstance(m, QuantizedVisionTransformerForImageClassification)
    assert sum(isinstance(x, QCustomLinearTorch) for x in m.modules()) == 73
    with pytest.raises(ValueError):
        build_model("bert", None, cfg)
