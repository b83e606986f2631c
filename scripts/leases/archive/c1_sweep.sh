# C1 (100k points, both parties): engine / prefix-depth sweep.  bash scripts/leases/c1_sweep.sh
set -o pipefail
O=gpurun_out/c1
mkdir -p $O
for cfg in "0 -1" "4 0" "4 10" "4 12" "4 14" "4 16" "1 0" "0 12"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --workload c1 --steps 20 --warmup 3 --no-cpu --no-compare --eval-mode $1 --prefix $2 > $O/c1_$1_$2.log 2>&1 || exit 1
  echo $cfg $(tail -1 $O/c1_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))")
done
