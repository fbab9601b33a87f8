"""The validate driver end to end on the GPU: a tiny numeric-class image folder (and the
synthetic mode) through calibration -> fixed ranges -> approx evaluation -> scoring."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_validate_driver_on_image_folder(tmp_path):
    from PIL import Image

    from fp8_quantization_amd import imagenet as inet
    rng = np.random.default_rng(0)
    for split, n in (("train", 4), ("val", 10)):
        for cls in ("0", "1", "999"):
            os.makedirs(tmp_path / split / cls)
            for i in range(n // 3 + 1):
                Image.fromarray(rng.integers(0, 256, size=(70, 90, 3), dtype=np.uint8)).save(
                    tmp_path / split / cls / f"{i}.png")
    out = tmp_path / "res.json"
    inet.main(["--images-dir", str(tmp_path), "--arch", "resnet18", "--image-size", "64", "--batch-size", "4",
               "--num-workers", "0", "--output", str(out)])
    res = json.loads(out.read_text())
    assert res["images"] == 12 and 0.0 <= res["top_1_accuracy"] <= res["top_5_accuracy"] <= 1.0
    assert np.isfinite(res["loss"]) and res["images_per_s"] > 0


def test_validate_driver_synthetic_mobilenet(tmp_path):
    from fp8_quantization_amd import imagenet as inet
    out = tmp_path / "res.json"
    inet.main(["--synthetic", "8", "--arch", "mobilenet_v2", "--image-size", "64", "--batch-size", "4",
               "--num-workers", "0", "--output", str(out)])
    res = json.loads(out.read_text())
    assert res["images"] == 8 and res["data"].startswith("synthetic")
