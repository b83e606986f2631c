# r03z3: final round-3 tree (pipelined row gen) — GPU suite, smoke, C3 bench line as the driver runs it, lat bench, latency kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],4), d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload lat > $O/bench_lat.json 2> $O/bench_lat.err || { tail -20 $O/bench_lat.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_lat.json')); print('lat eval/gen us', round(d['eval_us'],1), round(d['gen_us'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o lat -- python3 bench.py --workload lat --steps 200 --warmup 20 > $O/lat_trace.log 2>&1 || { tail -20 $O/lat_trace.log; exit 1; }
echo done
