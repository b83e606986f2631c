# r05d: paired-slot tail with row 0 (t_0 = party) folded into the constant (N = 16: (9,2), 22 reads per
# 16 B of y instead of 24): LAMBDA >= 32 parity tests, C4 config test, C4 line, C4 kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda or prg32 or empty" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
timeout -k 10 600 python -u -m pytest tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k c4 > $O/pytest_c4.log 2>&1 || { tail -60 $O/pytest_c4.log; exit 1; }
tail -1 $O/pytest_c4.log
for i in 1 2; do
timeout -k 10 500 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/bench_c4_$i.json 2> $O/bench_c4_$i.err || { tail -20 $O/bench_c4_$i.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4_$i.json')); r=d['roofline']; print('c4', d['value'], r['frac'], d['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace_c4.json 2> $O/bench_trace_c4.err || { tail -20 $O/bench_trace_c4.err; exit 1; }
python scripts/trace_summary.py $O/trace_c4 --tail 12 > $O/prof_c4.md && rm -rf $O/trace_c4
head -12 $O/prof_c4.md
