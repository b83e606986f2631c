# C2 (N = 4, 2^24 points): shared-prefix depth sweep.  bash scripts/leases/c2_sweep.sh
set -o pipefail
O=gpurun_out/c2s
mkdir -p $O
for d in ${DEPTHS:-21 22 23 24 25 26}; do
  timeout -k 10 200 python bench.py --workload c2 --steps ${STEPS:-5} --warmup ${WARM:-2} --no-cpu --no-compare --prefix $d > $O/c2_$d.log 2>&1 || exit 1
  echo $d $(tail -1 $O/c2_$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e9,3), round(r['kernel_ms'],3), round(r['executed_blocks_per_eval'],2))")
done
