# A/B on the full-domain eval (N = 4, 2^32 outputs): default lib vs libdcf_hip_<v>.so, 2 rounds
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" "$@"; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload fd --steps 3 --warmup 1 --no-cpu > gpurun_out/$T/fd_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/fd_$v.json')); r=d['roofline']; print('fd', '${v:-default}', round(d['value']/1e9,2), round(r['frac'],4), round(r['kernel_ms'],2))"
done; done
