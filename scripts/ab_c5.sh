# A/B of multi-key key placement on C5: default lib (HK=11) vs HK=0 (all SGPR) vs HK=8
T=$1; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" _hk0 _hk8; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/$T/c5$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/c5$v.json')); r=d['roofline']; print('c5$v', round(d['value']/1e6,1), round(r['eval_only']['frac'],4), round(d['phases_ms']['eval_party0'],2))"
done; done
