"""Build the gfx950 HIP library libfp8approx.so in-tree (fp8_quantization_amd/lib/).

    python -m fp8_quantization_amd.build_native        # or via __graft_entry__.build()

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off is load-bearing: every
reference torch op rounds once, so no multiply may be fused into a following add unless the
kernel asks for it explicitly (__fmaf_rn where the fused result is exact).
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "fp8approx.hip")
DEPS = [SRC, os.path.join(HERE, "csrc", "fp8approx_device.h"), os.path.join(HERE, "csrc", "gemm_f8mx.h"), os.path.join(HERE, "csrc", "conv_tbx.h"), os.path.join(HERE, "csrc", "gemm_tt.h"), os.path.join(HERE, "csrc", "gemm_tt16.h"), os.path.join(HERE, "csrc", "gemm_oh.h"),
        os.path.join(HERE, "csrc", "gemm_dense.h"), os.path.join(HERE, "csrc", "gemm_v5mx.h"),
        os.path.join(ROOT, "include", "fp8approx.h")]
OUT_DIR = os.path.join(HERE, "lib")
OUT = os.path.join(OUT_DIR, "libfp8approx.so")
ARCH = os.environ.get("FP8A_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the fp8approx HIP library cannot be built")


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


EXTRA = os.environ.get("FP8A_HIPCC_FLAGS", "-fno-slp-vectorize").split()


def build(force=False, verbose=False, out=None, extra=None):
    out = out or OUT
    if not force and out == OUT and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
           "-Wall"] + (EXTRA if extra is None else extra) + ["-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
