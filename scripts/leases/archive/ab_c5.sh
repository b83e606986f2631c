# A/B on C5 (and C3 once as a control): default lib vs libdcf_hip_<v>.so, 2 rounds
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" "$@"; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/$T/c5_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/c5_$v.json')); r=d['roofline']; print('c5', '${v:-default}', round(d['value']/1e6,1), round(r['eval_only']['frac'],4), round(d['phases_ms']['eval_party0'],2))"
done; done
