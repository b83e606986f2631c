mkdir -p gpurun_out/r02z_gen
for rep in 1 2; do for v in "" _g1; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/r02z_gen/c5$v.json 2>/dev/null || exit 1
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload lat > gpurun_out/r02z_gen/lat$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r02z_gen/c5$v.json')); l=json.load(open('gpurun_out/r02z_gen/lat$v.json')); print('$v', round(d['value']/1e6,1), d['phases_ms'], round(l['gen_us'],1), round(l['eval_us'],1))"
done; done
