# A/B of the single-call latency workload (benches/dcf.rs) and C1: bash scripts/leases/ab_lat.sh <tag> _v...
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" "$@"; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload lat > gpurun_out/$T/lat$v.json 2>/dev/null || exit 1
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > gpurun_out/$T/c1$v.json 2>/dev/null || exit 1
  python -c "import json; l=json.load(open('gpurun_out/$T/lat$v.json')); d=json.load(open('gpurun_out/$T/c1$v.json')); print('${v:-default}', round(l['gen_us'],1), round(l['eval_us'],1), round(d['value']/1e6,1))"
done; done
