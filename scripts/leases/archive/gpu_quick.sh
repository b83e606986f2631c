# Quick GPU check: parity tests + bench per AES engine (no CPU baseline).
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for mode in ${MODES:-1 2}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --eval-mode $mode > $OUT/bench_mode$mode.log 2>&1 || { tail -20 $OUT/bench_mode$mode.log; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_mode$mode.log').read().splitlines()[-1]);print('mode $mode', d['value'], d['roofline']['kernel_ms'])"
done
