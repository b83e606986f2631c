# r04y2: C5 key-major CW digest with every load issued before the LDS stores (compile-time trip
# counts) at tiles 32 x 16 / 64 x 8 / 128 x 4 (keys x levels) vs the previous kernel: multi-key
# parity on the default build, C5 A/B (2 alternating runs), C5 trace of the default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04y2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "multikey or c5" > $O/pytest_mk.log 2>&1 || { tail -60 $O/pytest_mk.log; exit 1; }
tail -1 $O/pytest_mk.log
for rep in 1 2; do for v in kmold km3216 km648 km1284; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -20 $O/c5_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); r=d['roofline']; print('c5 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4), round(r['eval_only']['frac'],4))"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o trace -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > $O/bench_trace_c5.json 2> $O/bench_trace_c5.err || { tail -20 $O/bench_trace_c5.err; exit 1; }
python scripts/trace_summary.py $O/trace_c5 --tail 12 > $O/prof_c5.md && rm -rf $O/trace_c5
head -10 $O/prof_c5.md
