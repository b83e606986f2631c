# A/B of tail work ranges on C4: default lib vs DCF_TAIL_ROUNDS variants (built as libdcf_hip_tr<R>.so)
T=$1; shift; mkdir -p gpurun_out/$T
for rep in 1 2; do for v in "" "$@"; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload c4 --steps ${STEPS:-10} --warmup 3 --no-cpu > gpurun_out/$T/c4$v.json 2> gpurun_out/$T/c4$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/c4$v.json')); r=d['roofline']; print('c4$v', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],2))"
done; done
