# A/B of kernel variants over several workloads: default lib vs libdcf_hip_<v>.so for each v.
# Usage (GPU box): WL="c3 c2 c5" REPS=2 bash scripts/leases/ab_multi.sh <tag> <v>...
set -o pipefail
T=$1; shift; mkdir -p gpurun_out/$T
for rep in $(seq ${REPS:-2}); do for w in ${WL:-c3 c2}; do for v in "" "$@"; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu --no-compare > gpurun_out/$T/${w}_${v}_$rep.json 2>gpurun_out/$T/${w}_${v}_$rep.err || { tail -5 gpurun_out/$T/${w}_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/$T/${w}_${v}_$rep.json').read().splitlines()[-1]); r=d.get('roofline') or {}; print('$w', '${v:-default}', round(d['value']/1e6,2), r.get('frac') and round(r['frac'],4), r.get('kernel_ms') and round(r['kernel_ms'],3), round(d['ms_per_step'],3))"
done; done; done
