# r04x: wide prefix build with A-D in one 4-block AES call (was two 2-block calls): wide parity,
# then a C4 line and its kernel trace (k_wpfx_build avg vs 0.396 ms in r04w).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wide or c4" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('c4', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu > $O/bench_trace_c4.json 2> $O/bench_trace_c4.err || { tail -20 $O/bench_trace_c4.err; exit 1; }
python scripts/trace_summary.py $O/trace_c4 --tail 12 > $O/prof_c4.md && rm -rf $O/trace_c4
head -10 $O/prof_c4.md
