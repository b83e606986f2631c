set -o pipefail
OUT=gpurun_out/${1:-hyb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for cfg in ${CFGS:-"1 6 1" "3 8 0" "3 9 0" "3 6 1" "3 7 1" "3 8 1" "3 9 1" "3 10 1" "3 11 1"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --eval-mode $1 --hybrid-split $2 --hybrid-mem $3 > $OUT/bench_$1_$2_$3.log 2>&1 || { tail -20 $OUT/bench_$1_$2_$3.log; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_$1_$2_$3.log').read().splitlines()[-1]);print('mode $1 split $2 mem $3', d['value'], d['roofline']['kernel_ms'])"
done
