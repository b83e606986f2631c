# bash scripts/leases/depth_sweep.sh <tag> <workload> <depths...>: bench at forced shared-prefix depths
T=$1; W=$2; shift 2
mkdir -p gpurun_out/$T
for d in "$@"; do
  timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 2 --no-cpu --no-compare --prefix $d > gpurun_out/$T/sweep_${W}_$d.json 2>gpurun_out/$T/sweep_${W}_$d.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/$T/sweep_${W}_$d.json')); r=d['roofline']; print('$W D=$d', round(d['value']/1e6,1), round(r['frac'],3), round(r['kernel_ms'],3), round(r['executed_blocks_per_eval'],2))"
done
