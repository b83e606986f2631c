# GPU tests + default bench + extra workloads.  bash scripts/gpu_round.sh <tag> [workloads...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],3), round(r['executed_blocks_per_eval'],2), r['no_prefix'])"
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu > $O/bench_$w.log 2>&1 || { tail -20 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$w', round(d['value']/1e6,1), r.get('frac'), r.get('executed_blocks_per_eval'))"
done
