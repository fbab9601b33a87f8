set -o pipefail
O=gpurun_out/mr; mkdir -p $O
C="--arch resnet18 --batch 4 --steps 2 --warmup 1 --cal-batch 4 --bn-stats-batches 1 --no-cpu-baseline"
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --share-device --dump-logits $O/w2.npy $C > $O/w2.json 2> $O/w2.err || exit 1
timeout -k 10 300 python bench.py --shard-seed 0 --dump-logits $O/w1_0.npy $C > $O/w1_0.json 2> $O/w1_0.err || exit 1
timeout -k 10 300 python bench.py --shard-seed 0 --dump-logits $O/w1_0b.npy $C > $O/w1_0b.json 2> $O/w1_0b.err || exit 1
python - <<'PY'
import numpy as np
O = "gpurun_out/mr"
a = np.load(f"{O}/w2.npy.rank0.npz"); b = np.load(f"{O}/w1_0.npy.rank0.npz"); c = np.load(f"{O}/w1_0b.npy.rank0.npz")
print("w1 run-to-run logits equal:", np.array_equal(b["logits"], c["logits"]))
print("w2 rank0 vs w1 logits equal:", np.array_equal(a["logits"], b["logits"]))
for k in a.files:
    if k == "logits": continue
    if k not in b.files: print("missing in w1", k); continue
    if not np.array_equal(a[k], b[k]): print("differs", k, a[k].ravel()[:4], b[k].ravel()[:4])
for k in b.files:
    if k not in a.files: print("missing in w2", k)
PY
