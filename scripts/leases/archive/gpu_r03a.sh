# Round-3 first GPU check: full GPU suite, latency sweep of the column kernels vs variants, lat + C3 bench.
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for v in "" _nooct _bigoct; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python scripts/lat_sweep.py > $O/lat_sweep$v.json 2> $O/lat_sweep$v.err || { tail -20 $O/lat_sweep$v.err; exit 1; }
  cat $O/lat_sweep$v.json
done
timeout -k 10 300 python bench.py --workload lat > $O/bench_lat.json 2> $O/bench_lat.err || { tail -20 $O/bench_lat.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_lat.json')); print('lat', round(d['gen_us'],1), round(d['eval_us'],1), d['cpu_baseline'])"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],3), d['ms_per_step'])"
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 300 python scripts/clock_probe.py > $O/clock_probe.json 2> $O/clock_probe.err || { tail -20 $O/clock_probe.err; exit 1; }
python -c "import json; d=json.load(open('$O/clock_probe.json')); print({k: d[k] for k in ('c4_ms_per_step','c4','c3_ms_per_step','c3')}, d['amd_smi']['error'], len(d['amd_smi']['samples']))"
