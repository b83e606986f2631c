# A/B of C1 (100k points, both parties) between the default lib and variants (dcf_amd/libdcf_hip<v>.so)
#   bash scripts/leases/ab_c1.sh <tag> _v1 _v2 ...
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" "$@"; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload c1 --steps ${STEPS:-300} --warmup 100 --no-cpu --no-compare > gpurun_out/$T/c1$v.json 2> gpurun_out/$T/c1$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/c1$v.json')); r=d['roofline']; print('c1$v', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],4), r.get('prefix_levels'))"
done; done
