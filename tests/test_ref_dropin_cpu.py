"""The drop-in routes of INTEGRATION.md §3 against the reference's own model wrapper.

tests/ref_dropin_check.py builds the reference's QuantizedMobileNetV2 (unmodified, imported from
/root/reference through the golden generator's import shim) with this repo's operators, in a
subprocess (the shim patches torch factory functions):
  Option A -- ``approx.approx_calculation`` aliased to fp8_quantization_amd.approx_calculation;
  Option B -- the reference's hijackers with this repo's run_forward mixins bound onto them.
Checks: every conv is this repo's approx conv operator (mixin present), the classifier this
repo's approx linear, and the state dict has exactly the reference build's keys and shapes
(G8's recorded reference state, tests/golden/g8_mbv2.npz).  Skipped where the reference checkout
is absent (it never is on the GPU box's CPU suite -- this is a build-container check)."""
import json
import os
import subprocess
import sys

import pytest

from tests import golden_io as gio

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "approx")), reason="reference checkout not mounted")
@pytest.mark.parametrize("route", ["A", "B"])
def test_reference_wrapper_builds_on_this_engine(route):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    out = subprocess.run([sys.executable, os.path.join(HERE, "ref_dropin_check.py"), route], capture_output=True,
                         text=True, timeout=600, env=env, cwd=os.path.dirname(HERE))
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    layers = res["layers"]
    convs = {k: v for k, v in layers.items() if k != "classifier.1"}
    assert len(convs) == 52, len(convs)  # MobileNetV2: 52 convs (17 depthwise) + the classifier
    assert sum(1 for v in convs.values() if v["groups"] > 1) == 17
    for name, v in convs.items():
        assert v["conv_mixin"] and v["module"] == "fp8_quantization_amd.approx_calculation", (name, v)
    assert layers["classifier.1"]["linear_mixin"], layers["classifier.1"]
    # the reference build's state-dict layout (G8 recorded it from the reference's own model)
    case = next(c for c in gio.meta()["g8"] if c["name"] == "mbv2_e4m3")
    g = gio.load("g8_mbv2.npz")
    ref = {k: list(g[f"mbv2_e4m3__state__{k}"].shape) for k in case["state_keys"]}
    assert res["state"] == ref
