# GPU tests + default bench + extra workloads.  bash scripts/leases/gpu_round.sh <tag> [workloads...]
# Each bench line is kept as gpurun_out/<tag>/bench_<w>.json.  NO_TESTS=1 skips pytest.
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  grep -E "test_config|PASS|FAIL" $O/pytest_gpu.log | grep test_config
fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 ${C3ARGS:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench_c3.json
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],3), round(r['executed_blocks_per_eval'],2), (d.get('host_path') or {}).get('value'), d.get('cpu_baseline',{}).get('value'))"
for w in "$@"; do
  # short steps (C1 ~1 ms, C2 ~4 ms) need a longer timed region: over a few ms the GPU clock is
  # still ramping after the warmup's sync (C2: 3 steps 4.10, 30 steps 4.68, 200 steps 4.71 G evals/s)
  case $w in c1) SW="--steps 300 --warmup 100";; c2) SW="--steps 60 --warmup 20";; c4) SW="--steps 10 --warmup 3";; *) SW="--steps 3 --warmup 1";; esac
  timeout -k 10 400 python bench.py --workload $w $SW > $O/bench_$w.log 2>&1 || { tail -20 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log > $O/bench_$w.json
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d.get('roofline') or {}; print('$w', round(d['value']/1e6,1), r.get('frac'), r.get('executed_blocks_per_eval'), d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline_1core',{}).get('value'), (d.get('host_path') or {}).get('value'))"
done
