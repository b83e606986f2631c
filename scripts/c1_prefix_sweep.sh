# Forced shared-prefix depth on the small-batch pair path (bench.py --workload c1 shape, one key):
#   bash scripts/c1_prefix_sweep.sh TAG "N..." "POINTS..." "OFFSETS..."   (depth = floor(log2 points) + offset; -1 = auto)
# One line per (N, points, depth) in gpurun_out/TAG/sweep.txt: ms per step (both parties) and evals/s.
T=$1; NS=${2:-16}; MS=${3:-"40000 100000 250000 500000"}; OFFS=${4:-"-1 1 2 3"}
mkdir -p gpurun_out/$T
for n in $NS; do for m in $MS; do
  lg=$(python -c "import math; print(int(math.log2($m)))")
  for o in auto $OFFS; do
    if [ $o = auto ]; then p=-1; else p=$((lg + o)); fi
    [ $p -ge $((8 * n)) ] && continue
    timeout -k 10 120 python bench.py --workload c1 --n-bytes $n --points $m --prefix $p --steps 100 --warmup 30 --no-cpu \
      --no-compare > gpurun_out/$T/c1_${n}_${m}_${p}.json 2> gpurun_out/$T/err.txt || { tail -5 gpurun_out/$T/err.txt; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$T/c1_${n}_${m}_${p}.json')); print('N=$n m=$m prefix=$p', round(d['ms_per_step'], 4), '%.4g' % d['value'])" | tee -a gpurun_out/$T/sweep.txt
  done
done; done
