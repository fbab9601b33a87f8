"""N > 1 ranks rehearsed on the one leased GPU (the 8-GPU node is the driver's).

`bench.py --gpus 2 --dist-backend gloo --share-device` runs the real multi-rank flow -- ranks
spawned by bench.py itself before any GPU call, per-rank library state (flag arenas, word images,
options) in two processes on cuda:0, rank-0-only calibration with the model-state and FP8-range
broadcasts, each rank's forward captured into a HIP graph in thread_local mode while the process
group is live, one logits all-gather per step -- with gloo's host-staged collectives standing in for
RCCL (which wants one GPU per rank).  The gathered logits must equal, bit for bit, two world-1 runs
on the same two input shards (--shard-seed), i.e. sharding changes nothing but where images run.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (no BN-statistics estimation: it runs the float model on MIOpen, whose algorithm choice -- and so
# the last bits of the statistics -- may differ between processes sharing the GPU; the state
# broadcast makes the ranks agree, but a separate world-1 process would then calibrate another model)
COMMON = ["--arch", "resnet18", "--batch", "4", "--steps", "2", "--warmup", "1", "--cal-batch", "4",
          "--bn-stats-batches", "0", "--no-cpu-baseline"]


def _bench(args, timeout=420):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(1200)
def test_bench_two_ranks_on_one_gpu_match_world1_shards(tmp_path):
    two = str(tmp_path / "w2.npy")
    line = _bench(["--gpus", "2", "--dist-backend", "gloo", "--share-device", "--dump-logits", two] + COMMON)
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 8 and line["config"]["parallelism"] == "dp2"
    hg = line["hip_graph"]
    assert hg["captured"] and hg["all_ranks_captured"] and hg["replay_matches_eager_bitwise"], json.dumps(hg)
    assert line["value"] > 0
    shards = []
    for r in (0, 1):
        p = str(tmp_path / f"w1_{r}.npy")
        one = _bench(["--shard-seed", str(r), "--dump-logits", p] + COMMON)
        assert one["n_gpus"] == 1 and one["hip_graph"]["captured"]
        shards.append(np.load(p))
    got = np.load(two)
    want = np.concatenate(shards)
    assert got.shape == want.shape == (8, 1000)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), "sharded logits differ from the world-1 runs"
