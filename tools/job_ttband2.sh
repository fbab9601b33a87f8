set -o pipefail
R=$(pwd); O=$R/gpurun_out/ttb2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for b in 0 1; do
  FP8A_TT_BAND=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/t$b -o run -- \
    python $R/bench.py --arch resnet50 --expo-width 2 --mant-width 5 --batch 512 --no-cpu-baseline --steps 3 --warmup 1 --no-graph > $O/t$b.log 2>&1 || exit 1
  cd $R && python tools/trace_breakdown.py $(ls $O/t$b/*kernel_trace.csv) --forwards 5:3 --out $O/bd$b.txt > /dev/null || exit 1
  sed -n 1,8p $O/bd$b.txt; cd /tmp
done
