# r03h: C2 next-point slot A/B: default (none) vs pfn2 (x word only) vs pfn1 (x + row), parity of pfn2 first
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_pfn2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c2 or eval_random or prefix or large_sample or dist" > $O/pytest_pfn2.log 2>&1 || { tail -30 $O/pytest_pfn2.log; exit 1; }
tail -1 $O/pytest_pfn2.log
for rep in 1 2 3; do for v in "" pfn2 pfn1; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 --no-cpu --no-compare > $O/c2_$v$rep.json 2> $O/c2_$v$rep.err || { tail -5 $O/c2_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$v$rep.json')); r=d['roofline']; p=d.get('phases',{}); print('c2', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3), round(p.get('table_ms',0),3), round(p.get('walk_ms',0),3))"
done; done
