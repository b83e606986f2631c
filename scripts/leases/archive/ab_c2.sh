# A/B on C2 (and C3 once): default lib vs libdcf_hip_<v>.so
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2 3; do for v in "" "$@"; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 3 --no-cpu --no-compare > gpurun_out/$T/c2_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/c2_$v.json')); r=d['roofline']; print('c2', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3))"
done; done
