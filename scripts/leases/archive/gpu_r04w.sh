# r04w: t-vector repack with 16-byte row loads (tvn) vs per-word conditional loads (tvo): wide
# parity on the default build, then C4 A/B, three alternating same-box runs, and a C4 trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wide or c4" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
for rep in 1 2 3; do for v in tvo tvn; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu > $O/bench_trace_c4.json 2> $O/bench_trace_c4.err || { tail -20 $O/bench_trace_c4.err; exit 1; }
python scripts/trace_summary.py $O/trace_c4 --tail 12 > $O/prof_c4.md && rm -rf $O/trace_c4
head -10 $O/prof_c4.md
