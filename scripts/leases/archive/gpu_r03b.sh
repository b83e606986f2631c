# Round-3 second check: GPU suite, latency sweep (thresholds), lat / C1 / C5 / C3 benches, clock probe (two methods).
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for v in "" _bigoct; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python scripts/lat_sweep.py > $O/lat_sweep$v.json 2> $O/lat_sweep$v.err || { tail -20 $O/lat_sweep$v.err; exit 1; }
  cat $O/lat_sweep$v.json
done
timeout -k 10 300 python bench.py --workload lat > $O/bench_lat.json 2> $O/bench_lat.err || { tail -20 $O/bench_lat.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_lat.json')); print('lat', round(d['gen_us'],1), round(d['eval_us'],1))"
for v in "" _bigoct; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > $O/bench_c1$v.json 2> $O/bench_c1$v.err || { tail -20 $O/bench_c1$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_c1$v.json')); print('c1$v', round(d['value']/1e6,1), d['roofline']['frac'], d['ms_per_step'])"
done
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; print('c5', round(d['value']/1e6,1), round(r['frac'],3), r['eval_only'], d['phases_ms'])"
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 400 python scripts/clock_probe.py > $O/clock_probe.json 2> $O/clock_probe.err || { tail -20 $O/clock_probe.err; exit 1; }
python -c "import json; d=json.load(open('$O/clock_probe.json')); print({k: d[k] for k in ('c4_ms_per_step','c4','c3_ms_per_step','c3')}); print(d['amd_smi_c4']); print(d['amd_smi_c3'])"
bash scripts/leases/gpu_c3_lease.sh r03b_c3
