# Parity tests + bench sweep over AES engine configs.
# CFGS="mode,split,mem mode,split,mem ..." (default below).
set -o pipefail
OUT=gpurun_out/${1:-hyb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for cfg in ${CFGS:-1,6,1 3,8,0 3,10,1 3,11,1 3,12,1}; do
  IFS=, read -r mode split mem <<< "$cfg"
  log=$OUT/bench_${mode}_${split}_${mem}.log
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --eval-mode $mode --hybrid-split $split --hybrid-mem $mem > $log 2>&1 || { tail -20 $log; exit 1; }
  python -c "import json;d=json.loads(open('$log').read().splitlines()[-1]);print('mode $mode split $split mem $mem', d['value'], d['roofline']['kernel_ms'])"
done
