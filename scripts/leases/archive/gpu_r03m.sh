# r03m: B-reuse chain without the word fetch (DCF_REUSE_CHAIN=2, single key) — GPU suite on it, then C3 / C2 A/B vs default
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_chain2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_chain2.log 2>&1 || { tail -30 $O/pytest_chain2.log; exit 1; }
tail -1 $O/pytest_chain2.log
for rep in 1 2 3; do for v in "" chain2; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-compare > $O/c3_$v$rep.json 2> $O/c3_$v$rep.err || { tail -5 $O/c3_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c3_$v$rep.json')); r=d['roofline']; print('c3', '${v:-default}', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],2), round(r['executed_blocks_per_eval'],2))"
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 --no-cpu --no-compare > $O/c2_$v$rep.json 2> $O/c2_$v$rep.err || { tail -5 $O/c2_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$v$rep.json')); r=d['roofline']; print('c2', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3), round(r['executed_blocks_per_eval'],2))"
done; done
