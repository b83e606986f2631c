# r04f: GPU suite; C2 with the table build's depth-first tail claiming nodes per wave (3 runs + in-kernel
# timeline); the C3 headline line (driver-shaped) with its kernel trace and FETCH_SIZE / WRITE_SIZE / SQ
# passes in the same lease; a C5 kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 5 --no-cpu --no-compare > $O/c2_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c2_$rep.json')); r=d['roofline']; print('c2', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(r['frac'],4), d.get('phases'))"
done
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 300 python scripts/c2_timeline.py > $O/c2_timeline.json 2> $O/c2_timeline.err || { tail -30 $O/c2_timeline.err; exit 1; }
cat $O/c2_timeline.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], r['frac'], r['kernel_ms'])"
TRAFFIC="k_eval16_stream C3 268435456 16 16 26 17179869184" bash scripts/leases/gpu_profile_w.sh r04f c3 || exit 1
head -12 $O/prof_c3.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o trace -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --no-compare > $O/trace_c5.log 2>&1 || { tail -20 $O/trace_c5.log; exit 1; }
python scripts/trace_summary.py $O/trace_c5 --tail 10 > $O/prof_c5.md && rm -rf $O/trace_c5
head -12 $O/prof_c5.md
