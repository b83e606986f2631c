# r04b: C4 tail with per-wave dynamic 16-point blocks (LDS counter) vs the static split (libdcf_hip_base.so):
# wide parity tests, same-box A/B (2 rounds), kernel trace, the in-kernel timeline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "wide or c4 or lambda or mmo" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -2 $O/pytest_wide.log
for rep in 1 2; do for v in base new; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ $v = base ] && L=$PWD/dcf_amd/libdcf_hip_base.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_c4_trace.json 2> $O/bench_c4_trace.err || { tail -30 $O/bench_c4_trace.err; exit 1; }
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 300 python scripts/c4_timeline.py > $O/c4_timeline.json 2> $O/c4_timeline.err || { tail -30 $O/c4_timeline.err; exit 1; }
cat $O/c4_timeline.json
