set -o pipefail
O=gpurun_out/shy
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "stream_hybrid" -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for cfg in "0xFFFF 0" "0x7777 0" "0x7777 1" "0xEEEE 1" "0x3333 0" "0x3333 1" "0xFFF0 1"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-compare --eval-mode 5 --shy-mask $1 --shy-prio $2 > $O/c3_$1_$2.log 2>&1 || exit 1
  echo $cfg $(tail -1 $O/c3_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['roofline']['kernel_ms'],1))")
done
