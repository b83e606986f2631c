# C4 (lambda = 16384): wide shared-prefix depth sweep.  bash scripts/c4_sweep.sh
set -o pipefail
O=gpurun_out/c4
mkdir -p $O
for d in 0 16 19 21 22 24; do
  timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --prefix $d > $O/c4_$d.log 2>&1 || exit 1
  echo $d $(tail -1 $O/c4_$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e6,2), round(r['kernel_ms'],2), round(r['frac'],3), round(r['executed_blocks_per_eval'],1), r.get('prefix_levels'))")
done
