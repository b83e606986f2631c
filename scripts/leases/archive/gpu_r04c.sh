# r04c: spill-free bitsliced engine (s / v in slabs): GPU suite, then the C3 A/B of the stream engine
# against stream-hybrid splits (same box), and the stand-alone bitsliced engine's rate.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() {  # tag, extra args
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-compare "${@:2}" > $O/c3_$1.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c3_$1.json')); r=d['roofline']; print('$1', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(r['frac'],4))"
}
for rep in 1 2; do
  run stream_$rep
  run shy_fff0_p1_$rep --eval-mode 5 --shy-mask 0xFFF0 --shy-prio 1
  run shy_7777_p1_$rep --eval-mode 5 --shy-mask 0x7777 --shy-prio 1
  run shy_7777_p0_$rep --eval-mode 5 --shy-mask 0x7777 --shy-prio 0
  run shy_ffff_$rep --eval-mode 5 --shy-mask 0xFFFF
done
run bs_2e26 --eval-mode 2 --points 67108864
