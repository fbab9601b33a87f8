"""Build the gfx950 HIP library libfp8approx.so in-tree (fp8_quantization_amd/lib/).

    python -m fp8_quantization_amd.build_native [--force]   # or via __graft_entry__.build()

The library is several translation units (csrc/fp8approx.hip: the C-ABI, host dispatch and small
kernels; csrc/k_*.hip: the GEMM kernel families, some compiled once per part), compiled in
parallel by hipcc and linked into one shared object.

Every build first copies the sources into a private snapshot directory and compiles from there:
hipcc reads a source once per offload pass (device, then host), so a source edited while a build
ran could give a host pass that registers a kernel its device pass never compiled -- the round-4
`Cannot find Symbol ... v5mx_decode_b` abort.  tests/test_abi_cpu.py checks the
built library for exactly that: every kernel the host side registers has a `.kd` symbol in the
gfx950 code object.

-ffp-contract=off is load-bearing: every reference torch op rounds once, so no multiply may be
fused into a following add unless the kernel asks for it explicitly (__fmaf_rn where the fused
result is exact).
"""
import concurrent.futures
import glob
import os
import shutil
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HEADER = os.path.join(ROOT, "include", "fp8approx.h")
OUT_DIR = os.path.join(HERE, "lib")
OUT = os.path.join(OUT_DIR, "libfp8approx.so")
ARCH = os.environ.get("FP8A_OFFLOAD_ARCH", "gfx950")
# (source, extra defines): one object per entry
UNITS = [("fp8approx.hip", [])] + [("k_fast.hip", [f"-DFP8A_FAST_PART={p}"]) for p in range(4)] + \
        [("k_f8mx.hip", [f"-DFP8A_XF_PART={p}"]) for p in range(3)] + [("k_tt.hip", []), ("k_v5.hip", [])]


def deps():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip"))) + [HEADER]


DEPS = deps()


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the fp8approx HIP library cannot be built")


def up_to_date(out=OUT):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in deps())


EXTRA = os.environ.get("FP8A_HIPCC_FLAGS", "-fno-slp-vectorize").split()


def _jobs():
    n = os.environ.get("MAX_JOBS") or os.environ.get("FP8A_BUILD_JOBS")
    if n:
        return max(1, int(n))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, len(UNITS), 16))


def build(force=False, verbose=False, out=None, extra=None):
    out = out or OUT
    if not force and up_to_date(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wall"] + \
            (EXTRA if extra is None else extra)
    t0 = time.time()  # the snapshot's time: a source edited after it leaves the library stale
    with tempfile.TemporaryDirectory(prefix="fp8a_build_") as tmp:
        # the snapshot keeps the sources' relative layout (csrc/*.hip include ../../include/fp8approx.h)
        src = os.path.join(tmp, "fp8_quantization_amd", "csrc")
        shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("*.o", "*.so"))
        os.makedirs(os.path.join(tmp, "include"))
        shutil.copy2(HEADER, os.path.join(tmp, "include", "fp8approx.h"))

        def compile_unit(i):
            name, defs = UNITS[i]
            obj = os.path.join(tmp, f"u{i}.o")
            cmd = [hipcc()] + flags + defs + ["-c", "-o", obj, os.path.join(src, name)]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {name} {' '.join(defs)}:\n{r.stderr[-4000:]}")
            return obj

        with concurrent.futures.ThreadPoolExecutor(_jobs()) as ex:
            objs = list(ex.map(compile_unit, range(len(UNITS))))
        tmp_out = os.path.join(tmp, "lib.so")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_out] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        shutil.copy2(tmp_out, out + ".tmp")
        os.replace(out + ".tmp", out)
    os.utime(out, (t0, t0))
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
