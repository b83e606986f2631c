# r03g: C2 next-point slot (PFN, default) — GPU suite on the default lib, then C2 A/B vs nopfn, C3 check
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do for v in "" nopfn; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 --no-cpu --no-compare > $O/c2_$v$rep.json 2> $O/c2_$v$rep.err || { tail -5 $O/c2_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$v$rep.json')); r=d['roofline']; p=d.get('phases',{}); print('c2', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3), round(p.get('table_ms',0),3), round(p.get('walk_ms',0),3))"
done; done
timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c2.json')); r=d['roofline']; print('c2 full', d['value'], r['frac'], d['cpu_baseline']['matches_gpu'])"
