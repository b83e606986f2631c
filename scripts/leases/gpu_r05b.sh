# r05b (r05a with the test fix): first tree of round 5 (retired bitsliced / hybrid engines, bench.py self-spawn + multi-GPU ABI
# check, C5 N > 1 check, ADVICE r04 fixes, scratch-free wide gen): GPU suite, smoke, C3 and C4 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],4), d['ms_per_step'])"
timeout -k 10 500 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4.json')); r=d['roofline']; print('c4', d['value'], r['frac'], d['ms_per_step'])"
