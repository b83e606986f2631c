# r04k: C1 (100k points, both parties) on the pair kernel (auto) vs the stream engine (--eval-mode 4,
# with its auto shared-prefix table); 2 same-box runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
for rep in 1 2; do for m in 0 4; do
  timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --eval-mode $m --no-cpu --no-compare > $O/c1_m${m}_$rep.json 2> $O/c1_m${m}_$rep.err || { tail -20 $O/c1_m${m}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_m${m}_$rep.json')); r=d['roofline']; print('c1 mode $m', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(r['frac'],4), r.get('engine'), r.get('executed_blocks_per_eval'))"
done; done
