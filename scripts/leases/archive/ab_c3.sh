# A/B on C3 and C2: default lib vs libdcf_hip_<v>.so, 2 rounds (timing only: --no-compare)
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" "$@"; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  for w in c3 c2; do
    DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu --no-compare > gpurun_out/$T/${w}_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/$T/${w}_$v.json')); r=d['roofline']; print('$w', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3))"
  done
done; done
